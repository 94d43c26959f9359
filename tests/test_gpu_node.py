"""GPU parity of one RaftServer spread over several shards (rh_node_create_devices): 4 and 8 shards
on device 0 -- the routing, event gathering, watch levels and lease bitmap an 8-GPU server runs,
exercised on a one-GPU box (every shard has its own context, stream and resident table).

Placement follows RaftServerProxy's divisions keyed by RaftGroupId (RaftServerProxy.java:89-150)
sharded by floorMod(UUID.hashCode(), n) (RaftId.hashCode, RaftId.java:119-122); each shard's state
is checked against tests/table_model.py (FollowerInfo / LeaderStateImpl replay over the oracle's
commit rule) in node-slot space, and the lease bitmap against the oracle's literal
LeaderStateImpl.hasLease / LeaderLease restatement (orc_lease_soa)."""
import numpy as np
import pytest

from tests.table_model import COL_COMMITTED, COL_FLUSH, TableModel
from tests.test_gpu_table import conf_word, random_deltas

pytestmark = pytest.mark.gpu

MS = 1_000_000
TIMEOUT = 100


@pytest.mark.parametrize("n_shards", [4, 8])
def test_node_shards_on_one_gpu(ctx, orc, n_shards):
    from ratis_amd import groups, shard
    rng = np.random.default_rng(100 + n_shards)
    cap = 1200
    n_groups = 3000
    msb, lsb = shard.random_group_ids(n_groups, seed=40 + n_shards)
    sh = shard.shard_of(msb, lsb, n_shards)                    # numpy restatement of UUID.hashCode
    with groups.RaftNode(0, cap, devices=[0] * n_shards) as node:
        assert node.n_shards == n_shards
        # placement: the library's floorMod(UUID.hashCode(), n) equals the restatement, and every
        # shard receives its groups in order
        fill = np.zeros(n_shards, dtype=np.int64)
        slots = np.empty(n_groups, dtype=np.int64)
        for i in range(n_groups):
            assert groups.shard_of(int(msb[i]), int(lsb[i]), n_shards) == sh[i]
            slots[i] = node.place(int(msb[i]), int(lsb[i]), int(fill[sh[i]]))
            fill[sh[i]] += 1
        assert fill.max() <= cap and (np.bincount(sh, minlength=n_shards) > 0).all()
        model = TableModel(n_shards * cap)
        shapes = [(0b1111, None), (0b111, None), (0b110011, 0b1111), (0b11, None), (0b1111111, None)]
        confs = np.zeros(n_shards * cap, dtype=np.uint32)
        for i, s in enumerate(slots):
            m = shapes[i % len(shapes)]
            c = conf_word(m[0], old_mask=m[1])
            base = int(rng.integers(1 << 20, 1 << 36))
            args = (int(s), c, base, base - int(rng.integers(0, 3000)), base - int(rng.integers(-200, 2000)))
            node.start(*args)
            model.start(*args)
            confs[s] = c
        for step in range(4):
            if step == 2:  # a conf change that moves slots across tiers on every shard
                for s in slots[::9]:
                    c = conf_word(0b11111, old_mask=0b111)
                    node.reconf(int(s), c, list(range(5)) + [-1])
                    model.reconf(int(s), c, list(range(5)) + [-1])
                    confs[s] = c
            d = random_deltas(rng, model, slots, 15000, set_frac=0.1 if step == 1 else 0.0)
            node.push(d)                                        # split by shard inside the library
            model.apply(d)
            adv, wall = node.update_commit(n_shards * cap)
            a_s, a_c, w_s, w_m = model.commit_batch(orc)
            assert np.array_equal(adv["slot"].astype(np.int64), a_s) and np.array_equal(adv["value"], a_c)
            assert np.array_equal(wall["slot"].astype(np.int64), w_s) and np.array_equal(wall["value"], w_m)
            assert a_s.size > 100 and len(set(a_s // cap)) == n_shards    # every shard contributed
            # commitIndexChanged per shard (the module's watchLevels pump), gathered in node slots
            evs = []
            for k, tab in enumerate(node.tables):
                ev = tab.commit_index_changed()
                ev_slots = ev["slot"].astype(np.int64) + k * cap
                evs.append((ev_slots, ev))
            got_s = np.concatenate([e[0] for e in evs])
            got = np.concatenate([e[1] for e in evs])
            m_s, m_lev, m_valid = model.watch(orc)
            o = np.argsort(got_s, kind="stable")
            assert np.array_equal(got_s[o], m_s)
            assert np.array_equal(got["min"][o], m_lev[0]) and np.array_equal(got["majority"][o], m_lev[1])
            assert np.array_equal(got["max"][o], m_lev[2]) and np.array_equal(got["valid"][o].astype(bool), m_valid)
            # resident columns of every shard = the model's rows of that shard
            for col in (0, 3, 17, COL_FLUSH, COL_COMMITTED):
                want = model.column(col)
                for k, tab in enumerate(node.tables):
                    assert np.array_equal(tab.read(col), want[k * cap:(k + 1) * cap]), (col, k)

        # ---- lease bitmap over the node: LeaderLease per division, follower replies, hasLease
        T0 = 1 << 60
        enabled = np.zeros(n_shards * cap, dtype=bool)
        enabled[slots] = rng.random(n_groups) < 0.85
        ts = np.full((14, n_shards * cap), T0, dtype=np.int64)
        for s in slots:
            node.lease_start(int(s), T0, bool(enabled[s]))
        now = T0 + 60 * MS
        widths = np.array([node.tables[s // cap].tier_width(int(s % cap)) for s in range(n_shards * cap)])
        for k in range(7):
            sl = slots[(widths[slots] > k) & (rng.random(n_groups) < 0.6)]
            st = now - rng.integers(0, 3 * TIMEOUT * MS, size=sl.size)
            node.push(groups.make_deltas(sl, 48 + k, st, ops=1))
            ts[k, sl] = st
        got = node.lease_batch(now, TIMEOUT)
        en = np.zeros((confs.size + 63) // 64, dtype=np.uint64)
        for s in np.nonzero(enabled)[0]:
            en[s // 64] |= np.uint64(1) << np.uint64(s % 64)
        lease_in = np.full(confs.size, T0, dtype=np.int64)
        ref = orc.lease_soa(ts, confs, lease_in, now, TIMEOUT, enabled_bits=en)
        want = np.unpackbits(ref["has_lease_bits"].view(np.uint8), bitorder="little")[:confs.size].astype(bool)
        assert np.array_equal(got, want)
        assert 0 < got.sum() < n_groups and len(set(np.nonzero(got)[0] // cap)) == n_shards


def test_node_rejects_bad_devices():
    from ratis_amd import _lib, groups
    with pytest.raises(_lib.IllegalArgumentError):
        groups.RaftNode(0, 100, devices=[])
    with pytest.raises(_lib.IllegalArgumentError):
        groups.RaftNode(0, 100, devices=[0, 1 << 20])
