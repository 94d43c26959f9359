"""GPU parity of the leader lease on the resident group table (rh_group_lease_start,
RH_COL_TS / RH_COL_LEASE / RH_COL_LEASE_ON deltas, rh_lease_batch) against the oracle's literal
LeaderStateImpl.hasLease / LeaderLease.extend restatement (orc_lease_soa), step by step:

  * LeaderLease created with the leader (lease = now, enabled per config, every FollowerInfo's
    lastRespondedAppendEntriesSendTime = its creation time: LeaderLease.java:37-38,
    FollowerInfoImpl.java:58), then replies stamping the followers
    (FollowerInfoImpl.updateLastRespondedAppendEntriesSendTime, LogAppenderDefault.java:102);
  * extend() when the lease lapsed (majority of current and old confs within the timeout), the
    extended lease stored and used by the next batch;
  * step-down / leader-not-in-conf disabling the lease (getAndSetEnabled(false), LSI:478, 744, 1042);
  * a reconf adding a follower that has not been stamped yet (treated as never active) and moving
    the slot to a wider tier;
  * singleton groups (always valid once enabled)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SELF, TRANS, SELF_OLD, ACTIVE = 1 << 14, 1 << 15, 1 << 30, 1 << 31
MS = 1_000_000
TIMEOUT = 100
FAR = 1 << 61   # how old an unstamped follower looks to the oracle (never active, never selected)


def word(new_mask, old_mask=None, self_new=True, self_old=True):
    w = new_mask | (SELF if self_new else 0) | ACTIVE
    if old_mask is not None:
        w |= TRANS | (old_mask << 16) | (SELF_OLD if self_old else 0)
    return w & 0xFFFFFFFF


def oracle_batch(orc, confs, ts, lease, enabled, now):
    """ts: [14][n] (np.nan-free; unstamped = None handled by the caller)"""
    n = confs.size
    en = np.zeros((n + 63) // 64, dtype=np.uint64)
    for s in np.nonzero(enabled)[0]:
        en[s // 64] |= np.uint64(1) << np.uint64(s % 64)
    ref = orc.lease_soa(ts, confs, lease, now, TIMEOUT, enabled_bits=en)
    has = np.unpackbits(ref["has_lease_bits"].view(np.uint8), bitorder="little")[:n].astype(bool)
    return has, ref["lease"]


def test_table_lease_sequence(ctx, orc):
    from ratis_amd import _lib, groups
    rng = np.random.default_rng(77)
    n = 700
    masks = [(0b111, None), (0b1111, None), (0b11111, None), (0b1111, 0b11110), (0, None), (0b11, None),
             (0b111111, 0b1111), (0b1111, None)]
    confs = np.array([word(*masks[i % len(masks)], self_new=(i % 13 != 5)) for i in range(n)], dtype=np.uint32)
    T0 = (1 << 60)
    enabled = np.array([i % 7 != 0 for i in range(n)])
    ts = np.full((14, n), T0, dtype=np.int64)      # FollowerInfo creation time = the leader start
    with groups.RaftGroupTable(ctx, capacity=n) as tab:
        for s in range(n):
            tab.start(s, int(confs[s]), 100, 50, 10)
            tab.lease_start(s, T0, bool(enabled[s]))
        lease = np.full(n, T0, dtype=np.int64)
        widths = np.array([tab.tier_width(s) for s in range(n)])
        now = T0
        for step in range(4):
            now += rng.integers(20, 80) * MS
            # replies from a random subset of followers: send times in the last 3 timeouts
            for k in range(14):
                sl = np.nonzero((widths > k) & (rng.random(n) < 0.6))[0]
                if sl.size:
                    st = now - rng.integers(0, 3 * TIMEOUT * MS, size=sl.size)
                    tab.update_last_responded(sl, k, st)
                    ts[k, sl] = st
            if step == 2:  # step-down / leader not in the new conf: lease disabled
                off = rng.choice(n, size=40, replace=False)
                tab.set_lease_enabled(off, False)
                enabled[off] = False
            if step == 3:  # reconf: a new follower slot 5 (unstamped) joins some 4-wide groups
                grow = [s for s in range(n) if confs[s] == word(0b1111) and s % 3 == 0][:20]
                for s in grow:
                    new = word(0b111111)
                    tab.reconf(s, new, src=list(range(4)) + [-1, -1])
                    confs[s] = new
                    ts[4:6, s] = now - FAR
                    widths[s] = tab.tier_width(s)
                assert all(widths[s] == 6 for s in grow)
            got = tab.lease_batch(now, TIMEOUT)
            want, lease_out = oracle_batch(orc, confs, ts, lease, enabled, now)
            assert np.array_equal(got, want), f"step {step}: {np.nonzero(got != want)[0][:10]}"
            assert np.array_equal(tab.read(_lib.RH_COL_LEASE), lease_out), f"step {step}"
            lease = lease_out
            assert want.any() and not want.all()
        assert np.array_equal(tab.read(_lib.RH_COL_LEASE_ON).astype(bool), enabled)
        for k in (0, 3):
            col = tab.read(_lib.RH_COL_TS(k))
            have = widths > k
            assert np.array_equal(col[have], ts[k, have])


def test_table_lease_unstamped_follower_is_never_active(ctx, orc):
    """A follower added by reconf has no lastRespondedAppendEntriesSendTime until the module stamps
    it: with 2 of 4 followers unstamped and 2 active, a 5-voter conf (self + 4) has exactly 3 of 5
    -> majority; with 3 unstamped, no majority and no extension."""
    from ratis_amd import _lib, groups
    T0 = 1 << 60
    with groups.RaftGroupTable(ctx, capacity=4) as tab:
        for s in range(2):
            tab.start(s, word(0b11), 1, 1, 1)
            tab.lease_start(s, T0, True)
        now = T0 + 3 * TIMEOUT * MS   # the lease from the start has lapsed
        tab.update_last_responded([0, 0, 1, 1], 0, [now - MS] * 4)
        tab.update_last_responded([0, 1], 1, [now - MS, now - 5 * TIMEOUT * MS])
        for s in range(2):
            tab.reconf(s, word(0b1111), src=[0, 1, -1, -1])
        got = tab.lease_batch(now, TIMEOUT)
        assert got[0] and not got[1] and not got[2:].any()
        lease = tab.read(_lib.RH_COL_LEASE)
        # extended to the majority-ack time: the 2nd freshest of the 4 followers' send times (both
        # stamped ones at now - 1 ms)
        assert lease[0] == now - MS and lease[1] == T0


def test_table_lease_api_errors(ctx):
    from ratis_amd import _lib, groups
    with groups.RaftGroupTable(ctx, capacity=8) as tab:
        with pytest.raises(_lib.IllegalArgumentError):
            tab.lease_start(3, 1, True)          # stopped slot
        with pytest.raises(_lib.IllegalArgumentError):
            tab.lease_batch(1, -1)
        tab.start(0, word(0b11), 1, 1, 1)
        with pytest.raises(_lib.IllegalArgumentError):
            tab.update_last_responded([0], 2, [5])   # follower column outside the slot's tier


def test_node_lease_one_shard(ctx, orc):
    """rh_node forms over a one-GPU mask equal the table's bits at node slots."""
    from ratis_amd import groups
    T0 = 1 << 60
    with groups.RaftNode(1, 128) as node:
        confs = [word(0b111), word(0), word(0b1111, 0b111)]
        for s, c in enumerate(confs):
            node.start(10 + s, c, 1, 1, 1)
            node.lease_start(10 + s, T0, True)
        now = T0 + 3 * TIMEOUT * MS
        tab = node.tables[0]
        for k in range(4):
            tab.update_last_responded([10, 12], k, [now - MS, now - MS])
        got = node.lease_batch(now, TIMEOUT)
        assert got.size == 128
        assert list(np.nonzero(got)[0]) == [10, 11, 12]   # 11: singleton
