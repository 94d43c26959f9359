"""GPU parity of the resident group table (rh_groups_*, rh_node_*) against a host model that
replays the reference's FollowerInfo / LeaderStateImpl semantics with the oracle's commit
arithmetic (tests/table_model.py).  Every step compares the events the table reports
(advanced commits, watch-ALL changes, commitIndexChanged levels) and the resident columns.

Scenarios from the reference's reconfiguration and leader-change paths:
  * stable -> joint (old+new) -> new conf, with the slot moving tiers 4 -> 6 -> 4 follower
    columns (applyOldNewConf / replicateNewConf, LeaderStateImpl.java:624-633, 1064-1074);
  * a follower replaced into a recycled slot (new FollowerInfo at -1, FollowerInfoImpl.java:42-43,
    LogAppender restart LeaderStateImpl.java:704-724);
  * a leader change with a new term start (StartupLogEntry, LeaderStateImpl.java:296-301);
  * setSnapshotIndex lowering a matchIndex (FollowerInfoImpl.java:147-151), interleaved with
    updateToMax deltas in one push."""
import numpy as np
import pytest

from tests.table_model import COL_COMMITTED, COL_FLUSH, OP_MAX, OP_SET, TableModel, tier_width

pytestmark = pytest.mark.gpu

SELF, TRANS, SELF_OLD, ACTIVE = 1 << 14, 1 << 15, 1 << 30, 1 << 31


def conf_word(new_mask, old_mask=None, self_new=True, self_old=True):
    w = new_mask | (SELF if self_new else 0) | ACTIVE
    if old_mask is not None:
        w |= TRANS | (old_mask << 16) | (SELF_OLD if self_old else 0)
    return w & 0xFFFFFFFF


STATS = {"advanced": 0, "watch_all": 0, "watch": 0}


def compare(tab, model, orc, watch=True, columns=True):
    got = tab.update_commit()
    STATS["advanced"] += got.advanced_slots.size
    STATS["watch_all"] += got.watch_all_slots.size
    a_s, a_c, w_s, w_m = model.commit_batch(orc)
    assert np.array_equal(got.advanced_slots, a_s)
    assert np.array_equal(got.advanced_commit, a_c)
    assert np.array_equal(got.watch_all_slots, w_s)
    assert np.array_equal(got.watch_all_min, w_m)
    if watch:
        ev = tab.commit_index_changed()
        STATS["watch"] += ev.size
        m_s, m_lev, m_valid = model.watch(orc)
        assert np.array_equal(ev["slot"].astype(np.int64), m_s)
        assert np.array_equal(ev["min"], m_lev[0]) and np.array_equal(ev["majority"], m_lev[1])
        assert np.array_equal(ev["max"], m_lev[2]) and np.array_equal(ev["valid"].astype(bool), m_valid)
    if columns:
        for col in [0, 1, 5, 13, 16, 21, COL_FLUSH, COL_COMMITTED, 34, 35]:
            assert np.array_equal(tab.read(col), model.column(col)), col
    return got


def random_deltas(rng, model, slots, k, set_frac=0.0, fcommit=True):
    """k deltas over started slots: matchIndex advances (some stale), follower commitIndex,
    flush advances, and optionally setSnapshotIndex-style SETs that may lower a matchIndex."""
    from ratis_amd.groups import make_deltas
    s = rng.choice(slots, size=k)
    w = model.width[s]
    kind = rng.random(k)
    col = np.where(kind < 0.6, rng.integers(0, 14, k) % w,
                   np.where(kind < 0.8, 16 + rng.integers(0, 14, k) % w, COL_FLUSH)) if fcommit else \
        np.where(kind < 0.8, rng.integers(0, 14, k) % w, COL_FLUSH)
    base = np.where(col == COL_FLUSH, model.flush[s], np.where(col < 16, model.match[col % 16, s],
                                                                 model.fcommit[col % 16, s]))
    base = np.where(base < 0, model.commit[s], base)
    val = base + rng.integers(-40, 400, k)
    op = np.where((rng.random(k) < set_frac) & (col < 16), OP_SET, OP_MAX)
    val = np.where(op == OP_SET, base - rng.integers(0, 300, k), val)   # SET may go down
    return make_deltas(s, col, val, op)


def test_reconfiguration_lifecycle_matches_reference(ctx, orc):
    from ratis_amd import groups
    rng = np.random.default_rng(2024)
    n = 3000
    model = TableModel(n, gap=-1)
    for k in STATS:
        STATS[k] = 0
    with groups.RaftGroupTable(ctx, capacity=n, gap_threshold=-1) as tab:
        base = rng.integers(1 << 20, 1 << 30, n)
        stable = conf_word(0b1111)
        for s in range(n):   # leader start of every division (5 peers: self + followers 0..3)
            ts = int(base[s] - rng.integers(0, 500))
            tab.start(s, stable, int(base[s]), int(base[s] - 1000), ts)
            model.start(s, stable, int(base[s]), int(base[s] - 1000), ts)
        assert tab.tier_width(0) == 4
        slots = np.arange(n)
        for step in range(3):
            d = random_deltas(rng, model, slots, 20000)
            tab.push(d)
            model.apply(d)
            compare(tab, model, orc)

        # stable -> joint: peers 2, 3 leave, newcomers take follower slots 4, 5 (new FollowerInfos)
        joint = slots[: n // 2]
        jw = conf_word(0b110011, old_mask=0b1111)
        src = [0, 1, 2, 3, -1, -1]
        for s in joint:
            tab.reconf(int(s), jw, src)
            model.reconf(int(s), jw, src)
        assert tab.tier_width(0) == 6 and tab.tier_width(n - 1) == 4
        for step in range(3):
            d = random_deltas(rng, model, slots, 20000)
            tab.push(d)
            model.apply(d)
            compare(tab, model, orc)

        # joint -> new conf: followers 2, 3 gone; the module renumbers 4 -> 2, 5 -> 3
        newc = conf_word(0b1111)
        for s in joint:
            tab.reconf(int(s), newc, [0, 1, 4, 5])
            model.reconf(int(s), newc, [0, 1, 4, 5])
        assert tab.tier_width(0) == 4
        d = random_deltas(rng, model, slots, 20000)
        tab.push(d)
        model.apply(d)
        compare(tab, model, orc)

        # a follower replaced into a recycled slot: slot 3 gets a new FollowerInfo (index -1) while
        # its predecessor's high matchIndex must not count
        rec = slots[::7]
        for s in rec:
            tab.reconf(int(s), newc, [0, 1, 2, -1])
            model.reconf(int(s), newc, [0, 1, 2, -1])
        compare(tab, model, orc)
        assert (tab.read(3)[rec] == -1).all()

        # leader change: a new leadership term re-arms the slot with a new term start
        lead = slots[1::5]
        for s in lead:
            ts = int(model.flush[s] + 1)
            tab.start(int(s), newc, int(model.flush[s] + 5), int(model.commit[s]), ts)
            model.start(int(s), newc, int(model.flush[s] + 5), int(model.commit[s]), ts)
        compare(tab, model, orc)
        for step in range(2):
            d = random_deltas(rng, model, slots, 20000)
            tab.push(d)
            model.apply(d)
            compare(tab, model, orc)

        # setSnapshotIndex lowering matchIndex, mixed with updateToMax in the same push
        d = random_deltas(rng, model, slots, 20000, set_frac=0.3)
        assert (d["op"] == OP_SET).any()
        tab.push(d)
        model.apply(d)
        compare(tab, model, orc)

        # step down of some divisions: no more events from them
        for s in slots[::11]:
            tab.stop(int(s))
            model.stop(int(s))
        d = random_deltas(rng, model, np.nonzero(model.started)[0], 20000)
        tab.push(d)
        model.apply(d)
        compare(tab, model, orc)
    # every kind of event was produced along the way (the comparisons were not vacuous)
    assert STATS["advanced"] > 2 * n and STATS["watch_all"] > 5 * n and STATS["watch"] > 5 * n, STATS


def test_set_after_max_same_cell_in_one_push(ctx, orc):
    """Sequential semantics inside one push: MAX then SET to the same cell ends at the SET value
    (the push is cut there), SET then MAX ends at the max of both."""
    from ratis_amd import groups
    with groups.RaftGroupTable(ctx, capacity=4) as tab:
        model = TableModel(4)
        w = conf_word(0b11)
        for s in range(4):
            tab.start(s, w, 100, 10, 0)
            model.start(s, w, 100, 10, 0)
        d = groups.make_deltas([0, 0, 1, 1, 2, 2, 2, 3], [0, 0, 0, 0, 1, 1, 1, 0],
                               [90, 40, 40, 90, 50, 60, 20, 70],
                               [OP_MAX, OP_SET, OP_SET, OP_MAX, OP_SET, OP_SET, OP_MAX, OP_SET])
        tab.push(d)
        model.apply(d)
        assert list(tab.read(0)) == [40, 90, -1, 70]
        assert tab.read(1)[2] == 60
        compare(tab, model, orc)


@pytest.mark.parametrize("seed", [1, 2])
def test_table_fuzz_every_width(ctx, orc, seed):
    """Random lifecycles over every tier width: starts, conf changes with random carry-over /
    reset maps (moving slots across tiers), stops, re-starts, MAX/SET deltas, gap clamp."""
    from ratis_amd import groups
    rng = np.random.default_rng(seed)
    n, gap = 4000, 300
    model = TableModel(n, gap=gap)

    def rand_conf():
        F = int(rng.integers(1, 15))
        new = int(rng.integers(1, 1 << F))
        if rng.random() < 0.3:
            return conf_word(new, old_mask=int(rng.integers(0, 1 << F)), self_new=rng.random() < 0.9,
                             self_old=rng.random() < 0.9)
        return conf_word(new, self_new=rng.random() < 0.95)

    with groups.RaftGroupTable(ctx, capacity=n, gap_threshold=gap) as tab:
        for step in range(12):
            for s in rng.choice(n, size=400, replace=False):
                s = int(s)
                r = rng.random()
                if not model.started[s] or r < 0.1:
                    c = rand_conf()
                    b = int(rng.integers(1000, 1 << 40))
                    args = (s, c, b, b - int(rng.integers(0, 2000)), b - int(rng.integers(-500, 3000)))
                    tab.start(*args)
                    model.start(*args)
                elif r < 0.5:
                    c = rand_conf()
                    src = [int(x) for x in rng.integers(-1, 14, size=14)]
                    tab.reconf(s, c, src)
                    model.reconf(s, c, src)
                elif r < 0.55:
                    tab.stop(s)
                    model.stop(s)
            live = np.nonzero(model.started)[0]
            d = random_deltas(rng, model, live, 30000, set_frac=0.05 if step % 3 == 0 else 0.0)
            tab.push(d)
            model.apply(d)
            compare(tab, model, orc, columns=step % 4 == 3)
            widths = {tab.tier_width(int(s)) for s in live[:2000]}
            assert widths == {tier_width(int(model.conf[s])) for s in live[:2000]}


def test_zero_copy_ring_pipelined_with_async_commit(ctx, orc):
    """rh_deltas_acquire/submit written in place while the previous evaluation is in flight
    (rh_commit_batch_async / _wait), as the bench's delta-streaming leg runs it."""
    from ratis_amd import _lib, groups, workload
    rng = np.random.default_rng(33)
    tiers = workload.commit_snapshot(40_000, joint_frac=0.1, peers=5, seed=9)
    n = sum(t.n for t in tiers)
    model = TableModel(n)
    with groups.RaftGroupTable(ctx, capacity=n) as tab:
        first = 0
        for h in tiers:
            tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            model.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            first += h.n
        compare(tab, model, orc, watch=False)
        live = np.arange(n)
        prev = None
        for step in range(6):
            # both staging paths: up to 65536 deltas the apply reads the pinned slot in place, past it
            # the slot goes to HBM by DMA on the copy stream first
            k = int(rng.integers(1000, 60000)) if step % 2 == 0 else int(rng.integers(70_000, 150_000))
            d = random_deltas(rng, model, live, k, fcommit=False)
            ring = tab.acquire_deltas()
            assert ring.size == _lib.RH_DELTA_SLOT
            ring[: d.size] = d
            ring[d.size]["slot"] = n + 3          # ignored by the device: slot out of range
            ring[d.size]["column"] = 0
            ring[d.size]["value"] = 1 << 60
            tab.submit_deltas(d.size + 1)
            tk = tab.commit_async()
            if prev is not None:
                got = tab.commit_wait(prev[0])
                assert np.array_equal(got.advanced_slots, prev[1][0]) and np.array_equal(got.advanced_commit, prev[1][1])
                assert np.array_equal(got.watch_all_slots, prev[1][2]) and np.array_equal(got.watch_all_min, prev[1][3])
            model.apply(d)
            prev = (tk, model.commit_batch(orc))
        got = tab.commit_wait(prev[0])
        assert np.array_equal(got.advanced_slots, prev[1][0]) and np.array_equal(got.advanced_commit, prev[1][1])
        with pytest.raises(_lib.RatisHipError):
            tab.commit_wait(prev[0] - 3)          # superseded ticket
        tab.acquire_deltas()
        with pytest.raises(_lib.RatisHipError):
            tab.acquire_deltas()                  # one slot at a time
        with pytest.raises(_lib.RatisHipError):
            tab.push_deltas([1], [0], [1])        # push while a slot is acquired
        tab.submit_deltas(0)


def test_table_rejects_bad_input(ctx):
    from ratis_amd import _lib, groups
    with groups.RaftGroupTable(ctx, capacity=100) as tab:
        tab.start(5, conf_word(0b11), 10, 2, 0)
        with pytest.raises(_lib.IllegalArgumentError):
            tab.push_deltas([6], [0], [1])                    # slot never started
        with pytest.raises(_lib.IllegalArgumentError):
            tab.push_deltas([5], [2], [1])                    # column beyond the slot's width (2)
        with pytest.raises(_lib.IllegalArgumentError):
            tab.push_deltas([100], [0], [1])                  # slot out of range
        with pytest.raises(_lib.IllegalArgumentError):
            tab.push_deltas([5], [0], [1], ops=7)             # unknown op
        with pytest.raises(_lib.IllegalArgumentError):
            tab.start(100, conf_word(1), 1, 1, 1)             # slot out of range
        with pytest.raises(_lib.RatisHipError):
            tab.reconf(7, conf_word(1))                       # not started
        with pytest.raises(_lib.IllegalArgumentError):
            tab.reconf(5, conf_word(1), [99] + [0] * 13)      # bad src entry
        tab.update_match_index([5], 0, [9])
        tab.update_match_index([5], 1, [8])
        r = tab.update_commit()
        assert list(r.advanced_slots) == [5] and list(r.advanced_commit) == [9]   # sorted [8,9,10] -> 9
        assert list(r.watch_all_slots) == [5] and list(r.watch_all_min) == [8]
        r = tab.update_commit()                               # nothing dirty: no events
        assert r.advanced_slots.size == 0 and r.watch_all_slots.size == 0


def test_node_on_one_gpu(ctx, orc):
    """rh_node over the device mask of this box (one GPU: mask 0x1): placement by
    floorMod(RaftGroupId.hashCode(), 1), routing of starts / deltas, gathered events."""
    from ratis_amd import groups, shard
    rng = np.random.default_rng(5)
    cap = 2000
    with groups.RaftNode(0x1, cap) as node:
        assert node.n_shards == 1
        model = TableModel(cap)
        msb, lsb = shard.random_group_ids(500, seed=8)
        slots = [node.place(int(a), int(b), i) for i, (a, b) in enumerate(zip(msb, lsb))]
        assert slots == list(range(500))
        w = conf_word(0b111)
        for s in slots:
            node.start(s, w, 1000 + s, 10, 5)
            model.start(s, w, 1000 + s, 10, 5)
        d = random_deltas(rng, model, np.array(slots), 5000, fcommit=False)
        node.push(d)
        model.apply(d)
        adv, wall = node.update_commit(cap)
        a_s, a_c, w_s, w_m = model.commit_batch(orc)
        assert np.array_equal(adv["slot"].astype(np.int64), a_s) and np.array_equal(adv["value"], a_c)
        assert np.array_equal(wall["slot"].astype(np.int64), w_s) and np.array_equal(wall["value"], w_m)
