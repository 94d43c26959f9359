"""GPU parity of the resident table's event path (round 4): the evaluation kernels write their
records straight into the contiguous result lists, one range per workgroup, and the evaluation's
last workgroup publishes the list lengths (ratis_amd/csrc/rh_internal.h, TableEvents).  Checked
against tests/table_model.py (the reference's FollowerInfo / LeaderStateImpl semantics over the
oracle's commit arithmetic):

  * every sink (HOST_MAPPED: lists in pinned memory; DEVICE: lists in HBM + D2H in _wait; AUTO, the
    default: DEVICE for tile evaluations, HOST_MAPPED for list evaluations), for
    updateCommit (advanced + watch-ALL) and commitIndexChanged, on a table of 40+ workgroups;
  * sparse dirty sets, where most 128-row tiles are clean and skipped by their summary byte;
  * evaluations whose ticket is superseded without a wait, and an evaluation after them;
  * the async forms of commitIndexChanged and hasLease (rh_watch_levels_async / _wait,
    rh_lease_batch_async / _wait), their misuse, and the node forms over 4 shards on one GPU."""
import os

import numpy as np
import pytest

from tests.table_model import TableModel
from tests.test_gpu_table import compare, conf_word, random_deltas

pytestmark = pytest.mark.gpu


def _loaded(ctx, model, n, seed):
    from ratis_amd import groups, workload
    tiers = workload.commit_snapshot(n, joint_frac=0.1, peers=5, seed=seed)
    tab = groups.RaftGroupTable(ctx, capacity=sum(t.n for t in tiers))
    first = 0
    for h in tiers:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        if model is not None:
            model.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        first += h.n
    return tab, first


@pytest.mark.parametrize("sink", ["host_mapped", "device", "auto"])
def test_event_sinks_match_model(ctx, orc, sink):
    from ratis_amd import _lib
    rng = np.random.default_rng(404)
    n = 60_000   # 40+ workgroups of 1,536 rows, each taking its range of the lists
    model = TableModel(n)
    tab, n = _loaded(ctx, model, n, seed=41)
    try:
        tab.set_event_sink({"device": _lib.RH_EVENTS_DEVICE, "host_mapped": _lib.RH_EVENTS_HOST_MAPPED,
                            "auto": _lib.RH_EVENTS_AUTO}[sink])
        compare(tab, model, orc, columns=False)
        live = np.arange(n)
        for step, k in enumerate([n // 2, 3 * n, n // 100, 7, 0]):
            d = random_deltas(rng, model, live, k) if k else np.zeros(0, dtype=_lib_delta_dtype())
            tab.push(d)
            model.apply(d)
            got = compare(tab, model, orc, columns=step == 1)
            if k == 0:
                assert got.advanced_slots.size == 0 and got.watch_all_slots.size == 0
    finally:
        tab.close()


def _lib_delta_dtype():
    from ratis_amd.groups import DELTA_DTYPE
    return DELTA_DTYPE


def test_sparse_dirty_tiles_are_skipped_exactly(ctx, orc):
    """A few dirty rows in a large table: the clean tiles' waves return on their summary byte; the
    dirty rows (first / last row of a tile, both rows of one lane, the table's last tile) report."""
    from ratis_amd import groups
    rng = np.random.default_rng(9)
    n = 40_000
    model = TableModel(n)
    tab, n = _loaded(ctx, model, n, seed=3)
    try:
        compare(tab, model, orc, columns=False)
        for rows in ([0], [127, 128], [254, 255], [n - 1], list(rng.choice(n, 50, replace=False))):
            s = np.array(rows, dtype=np.int64)
            d = groups.make_deltas(s, np.zeros(s.size, np.int64), model.flush[s] + 1000)   # follower 0 jumps ahead
            d2 = groups.make_deltas(s, np.ones(s.size, np.int64), model.flush[s] + 1000)
            d = np.concatenate([d, d2])
            tab.push(d)
            model.apply(d)
            got = compare(tab, model, orc, columns=False)
            assert set(got.advanced_slots.tolist()) <= set(rows)
            r = tab.update_commit()                       # nothing dirty any more: no events
            assert r.advanced_slots.size == 0 and r.watch_all_slots.size == 0
            model.commit_batch(orc)
    finally:
        tab.close()


def test_superseded_tickets_do_not_leak_into_later_results(ctx, orc):
    """kEvSets + 1 evaluations in flight with only the last waited (the others superseded), then
    evaluations that are waited: every waited list equals the model's for its step."""
    from ratis_amd import _lib
    rng = np.random.default_rng(77)
    model = TableModel(30_000)
    tab, n = _loaded(ctx, model, 30_000, seed=5)
    try:
        compare(tab, model, orc, columns=False)
        live = np.arange(n)
        expect = None
        tickets = []
        for step in range(4):
            d = random_deltas(rng, model, live, 20_000, fcommit=False)
            tab.push(d)
            model.apply(d)
            tickets.append(tab.commit_async(watch_all=True))
            expect = model.commit_batch(orc)
        for tk in tickets[:-3]:
            with pytest.raises(_lib.RatisHipError):
                tab.commit_wait(tk)                       # its result set was reused
        got = tab.commit_wait(tickets[-1])
        assert np.array_equal(got.advanced_slots, expect[0]) and np.array_equal(got.advanced_commit, expect[1])
        assert np.array_equal(got.watch_all_slots, expect[2]) and np.array_equal(got.watch_all_min, expect[3])
        for step in range(3):
            d = random_deltas(rng, model, live, 5_000, fcommit=False)
            tab.push(d)
            model.apply(d)
            compare(tab, model, orc, watch=False, columns=False)
    finally:
        tab.close()


def test_async_watch_and_lease_forms(ctx, orc):
    from ratis_amd import _lib, groups
    rng = np.random.default_rng(12)
    model = TableModel(20_000)
    tab, n = _loaded(ctx, model, 20_000, seed=8)
    twin, _ = _loaded(ctx, None, 20_000, seed=8)
    try:
        with pytest.raises(_lib.RatisHipError):
            tab.watch_wait()                              # nothing in flight
        with pytest.raises(_lib.RatisHipError):
            tab.lease_wait()
        compare(tab, model, orc, watch=False, columns=False)
        twin.update_commit()
        live = np.arange(n)
        for step in range(3):
            d = random_deltas(rng, model, live, 8_000)
            tab.push(d)
            twin.push(d)
            model.apply(d)
            compare(tab, model, orc, watch=False, columns=False)
            twin.update_commit()
            tab.watch_async()
            ev = tab.watch_wait()
            m_s, m_lev, m_valid = model.watch(orc)
            assert np.array_equal(ev["slot"].astype(np.int64), m_s)
            assert np.array_equal(ev["min"], m_lev[0]) and np.array_equal(ev["max"], m_lev[2])
            assert np.array_equal(ev["majority"], m_lev[1]) and np.array_equal(ev["valid"].astype(bool), m_valid)
            assert np.array_equal(twin.commit_index_changed()["slot"], ev["slot"])
        # lease: async / wait against the blocking form on the twin fed the same stamps
        now = 1 << 50
        for s in range(0, n, 3):
            tab.lease_start(s, now, True)
            twin.lease_start(s, now, True)
        for k in range(3):   # 3 of 4 followers of every even slot reply late: a majority at 150 ms
            sl = np.arange(0, n, 2)
            st = now + 140_000_000 - rng.integers(0, 30_000_000, sl.size)
            tab.update_last_responded(sl, k, st)
            twin.update_last_responded(sl, k, st)
        for dt in (50_000_000, 150_000_000):
            tab.lease_async(now + dt, 100)
            a = tab.lease_wait()
            b = twin.lease_batch(now + dt, 100)
            assert np.array_equal(a, b) and a.any()
        tab.lease_async(now, 100)
        tab.lease_async(now + 1, 100)                     # a second batch replaces the first
        assert tab.lease_wait().shape == (tab.capacity,)
    finally:
        tab.close()
        twin.close()


def test_node_watch_levels_and_lease_over_four_shards(ctx, orc):
    from ratis_amd import groups
    rng = np.random.default_rng(21)
    cap = 3000
    with groups.RaftNode(0, cap, devices=[0, 0, 0, 0]) as node:
        models = [TableModel(cap) for _ in range(4)]
        for sh in range(4):
            for s in range(0, cap, 2):
                w = conf_word(int(rng.integers(1, 1 << 6)))
                node.start(sh * cap + s, w, 5000, 100, 50)
                models[sh].start(s, w, 5000, 100, 50)
        deltas = []
        for sh in range(4):
            d = random_deltas(rng, models[sh], np.arange(0, cap, 2), 4000)
            models[sh].apply(d)
            d = d.copy()
            d["slot"] += sh * cap
            deltas.append(d)
        node.push(np.concatenate(deltas))
        node.update_commit(4 * cap)
        for m in models:
            m.commit_batch(orc)
        ev = node.watch_levels(4 * cap)
        want = []
        for sh, m in enumerate(models):
            s, lev, valid = m.watch(orc)
            want.append(s + sh * cap)
        assert np.array_equal(ev["slot"].astype(np.int64), np.concatenate(want))
        assert node.watch_levels(4 * cap).size == 0       # nothing changed since
        bits = node.lease_batch(1 << 40, 100)             # no lease started: no division has one
        assert bits.shape == (4 * cap,) and not bits.any()


@pytest.mark.parametrize("seed,sink", [(3, "auto"), (4, "device")])
def test_list_and_tile_evaluations_interleaved(ctx, orc, seed, sink):
    """Sparse pushes run over the dirty-row lists (list mode), dense ones over every tile: steps of
    either kind, follower-commit-only steps (commitIndexChanged from the watch list), control ops
    (which give the lists up until the next evaluation) and the zero-copy ring, all against the
    model -- and both modes must actually run.  DEVICE runs every list evaluation in REGION mode
    (masks per wave and pass, records rebuilt from the list entries by the gather)."""
    from ratis_amd import _lib, groups
    rng = np.random.default_rng(seed)
    n = 50_000
    model = TableModel(n)
    tab, n = _loaded(ctx, model, n, seed=seed + 10)
    modes = {"commit": set(), "watch": set()}
    try:
        tab.set_event_sink({"device": _lib.RH_EVENTS_DEVICE, "auto": _lib.RH_EVENTS_AUTO}[sink])
        tab.set_timing(True)
        compare(tab, model, orc, columns=False)
        live = np.arange(n)
        for step in range(14):
            k = int(rng.choice([3, 40, 700, 1500, 20_000, 120_000]))
            if step % 5 == 4:   # follower commitIndex reports only
                s = rng.choice(live, size=min(k, 2000))
                col = 16 + rng.integers(0, 4, s.size)
                d = groups.make_deltas(s, col, model.commit[s] - rng.integers(0, 3, s.size))
            else:
                d = random_deltas(rng, model, live, k, fcommit=step % 2 == 0)
            if step == 7:       # a control op between pushes: lists given up, tiles evaluated
                w = conf_word(0b1111)
                tab.start(5, w, 10_000, 9_000, 8_000)
                model.start(5, w, 10_000, 9_000, 8_000)
            if step % 3 == 2:
                ring = tab.acquire_deltas()
                ring[: d.size] = d
                tab.submit_deltas(d.size)
            else:
                tab.push(d)
            model.apply(d)
            got = tab.update_commit()
            modes["commit"].add(tab.last_was_list())
            a_s, a_c, w_s, w_m = model.commit_batch(orc)
            assert np.array_equal(got.advanced_slots, a_s) and np.array_equal(got.advanced_commit, a_c), step
            assert np.array_equal(got.watch_all_slots, w_s) and np.array_equal(got.watch_all_min, w_m), step
            ev = tab.commit_index_changed()
            modes["watch"].add(tab.last_was_list())
            m_s, m_lev, m_valid = model.watch(orc)
            assert np.array_equal(ev["slot"].astype(np.int64), m_s), step
            assert np.array_equal(ev["min"], m_lev[0]) and np.array_equal(ev["majority"], m_lev[1]), step
            assert np.array_equal(ev["max"], m_lev[2]) and np.array_equal(ev["valid"].astype(bool), m_valid), step
        assert modes["commit"] == {True, False} and modes["watch"] == {True, False}, modes
        for col in [0, 1, 16, 32, 33]:
            assert np.array_equal(tab.read(col), model.column(col)), col
    finally:
        tab.close()


@pytest.mark.parametrize("sink", ["auto", "device"])
def test_list_mode_over_every_width(ctx, orc, sink):
    """List entries carry their tier ((tier << 28) | row) and a wave's lanes may hold rows of
    different widths: a table started over every width (1..14 followers, some in joint consensus)
    gets sparse pushes that run in list mode -- commit and commitIndexChanged -- against the model,
    with a control op between two of them (lists given up once, then list mode again)."""
    from ratis_amd import _lib, groups
    rng = np.random.default_rng(77)
    n = 4000
    model = TableModel(n)
    with groups.RaftGroupTable(ctx, capacity=n) as tab:
        tab.set_event_sink({"device": _lib.RH_EVENTS_DEVICE, "auto": _lib.RH_EVENTS_AUTO}[sink])
        tab.set_timing(True)
        for s in range(n):
            F = 1 + s % 14
            new = int(rng.integers(1, 1 << F))
            c = conf_word(new, old_mask=int(rng.integers(0, 1 << F))) if s % 5 == 0 else conf_word(new)
            b = int(rng.integers(1000, 1 << 40))
            args = (s, c, b, b - int(rng.integers(0, 2000)), b - int(rng.integers(-500, 3000)))
            tab.start(*args)
            model.start(*args)
        assert {tab.tier_width(s) for s in range(n)} == {2, 4, 6, 8, 10, 12, 14}
        compare(tab, model, orc, columns=False)          # after control ops: tile evaluations
        live = np.arange(n)
        modes = []
        # a push of k deltas bounds k markings of each kind, the commit evaluation k more for
        # commitIndexChanged: both lists hold while 2 k <= lcap = 1024 (4000 rows)
        for step, k in enumerate([5, 60, 400, 1000, 30, 450, 250]):
            if step == 4:
                tab.stop(17)
                model.stop(17)
                live = live[live != 17]
            d = random_deltas(rng, model, live, k)
            tab.push(d)
            model.apply(d)
            got = tab.update_commit()
            a_s, a_c, w_s, w_m = model.commit_batch(orc)
            assert np.array_equal(got.advanced_slots, a_s) and np.array_equal(got.advanced_commit, a_c), step
            assert np.array_equal(got.watch_all_slots, w_s) and np.array_equal(got.watch_all_min, w_m), step
            ml = tab.last_was_list()
            ev = tab.commit_index_changed()
            m_s, m_lev, m_valid = model.watch(orc)
            assert np.array_equal(ev["slot"].astype(np.int64), m_s), step
            assert np.array_equal(ev["min"], m_lev[0]) and np.array_equal(ev["majority"], m_lev[1]), step
            assert np.array_equal(ev["max"], m_lev[2]) and np.array_equal(ev["valid"].astype(bool), m_valid), step
            modes.append((ml, tab.last_was_list()))
        assert modes[3] == (True, False), modes              # 2 k > lcap: the watch list given up
        assert modes[4] == (False, False), modes             # the control op gave both lists up
        assert all(m == (True, True) for i, m in enumerate(modes) if i not in (3, 4)), modes
        for col in [0, 1, 7, 13, 16, 29, 32, 33]:
            assert np.array_equal(tab.read(col), model.column(col)), col


def test_list_region_mode_many_marks(ctx, orc):
    """AUTO list evaluations of at least 8192 marked rows run in REGION mode (groups.cpp evaluate):
    masks per wave and pass, the records rebuilt by the gather from the list entries.  On 1.5M
    rows (list capacity 46,875 per region) 45,000 deltas need two passes of the 480-wave list grid
    (3,840 entries per region and pass, ~4,500 updateCommit marks per region); 9,000 one pass; 500
    the pinned lists (counter mode).  Against the model, commit and commitIndexChanged."""
    rng = np.random.default_rng(515)
    n = 1_500_000
    model = TableModel(n)
    tab, n = _loaded(ctx, model, n, seed=51)
    try:
        tab.set_timing(True)
        compare(tab, model, orc, columns=False)   # after the load: tile evaluations
        live = np.arange(n)
        for k in (45_000, 9_000, 500, 45_000):
            d = random_deltas(rng, model, live, k)
            tab.push(d)
            model.apply(d)
            got = tab.update_commit()
            assert tab.last_was_list(), k
            a_s, a_c, w_s, w_m = model.commit_batch(orc)
            assert np.array_equal(got.advanced_slots, a_s) and np.array_equal(got.advanced_commit, a_c), k
            assert np.array_equal(got.watch_all_slots, w_s) and np.array_equal(got.watch_all_min, w_m), k
            ev = tab.commit_index_changed()
            m_s, m_lev, m_valid = model.watch(orc)
            assert np.array_equal(ev["slot"].astype(np.int64), m_s), k
            assert np.array_equal(ev["min"], m_lev[0]) and np.array_equal(ev["majority"], m_lev[1]), k
            assert np.array_equal(ev["max"], m_lev[2]) and np.array_equal(ev["valid"].astype(bool), m_valid), k
        for col in [0, 1, 16, 32, 33]:
            assert np.array_equal(tab.read(col), model.column(col)), col
    finally:
        tab.close()


def test_separate_done_word_of_large_tables(ctx, orc, monkeypatch):
    """28-bit list counts (tables of 2^24 rows and more) leave 8 bits of done count in the counter
    word: tile evaluations of more than 255 workgroups then count themselves on the separate done
    word (TableEvents.packed = 0).  Forced here on a 400k-row table (261 workgroups) through the
    library's test knob, with 3000 ten-follower groups beside config 3's so that both width
    classes launch (the second launch publishes)."""
    from ratis_amd import _lib, groups, workload
    monkeypatch.setenv("RATIS_HIP_TABLE_CNT_BITS", "28")
    rng = np.random.default_rng(28)
    tiers = workload.commit_snapshot(400_000, joint_frac=0.1, peers=5, seed=28)
    n0 = sum(t.n for t in tiers)
    n = n0 + 3000
    model = TableModel(n)
    tab = groups.RaftGroupTable(ctx, capacity=n)
    try:
        first = 0
        for h in tiers:
            tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            model.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            first += h.n
        w = conf_word(0b1111111111)
        for s_ in range(n0, n):
            tab.start(s_, w, 5000, 100, 50)
            model.start(s_, w, 5000, 100, 50)
        live = np.arange(n)
        for sink in (_lib.RH_EVENTS_AUTO, _lib.RH_EVENTS_HOST_MAPPED):
            tab.set_event_sink(sink)
            compare(tab, model, orc, columns=False)
            for k in (n, n // 10, 500):
                d = random_deltas(rng, model, live, k)
                tab.push(d)
                model.apply(d)
                compare(tab, model, orc, columns=False)
    finally:
        tab.close()


@pytest.mark.parametrize("sink", ["device", "auto"])
def test_region_records_survive_later_writers(ctx, orc, sink):
    """updateCommit in REGION mode writes no records: the gather rebuilds them behind the evaluation
    from the table's row-slot, commit and watch-ALL columns, and commitIndexChanged's from the
    row-slot and level columns (rh_internal.h, TableEvents), so every later writer of those columns
    must come after them (the table stream's order; with RH_GATHER_SIDE=1 the side stream's gathers
    and groups.cpp gather_fence / wgather_fence).  A commitIndexChanged evaluation with ~half a
    million changed levels goes first, so its record gather takes long (~16 MB across PCIe) and the
    updateCommit gather queues behind it; meanwhile the host
    rewrites every column that gather reads -- COMMITTED deltas on the advanced rows, stops, restarts
    with other commits, reconfigurations into another tier -- and starts a second evaluation.  Both
    tickets' lists must be what their evaluations computed."""
    from ratis_amd import _lib, groups
    rng = np.random.default_rng(1234)
    n = int(os.environ.get("RH_TEST_HAZARD_ROWS", 1_000_000))
    model = TableModel(n)
    tab, n = _loaded(ctx, model, n, seed=77)
    try:
        tab.set_event_sink({"device": _lib.RH_EVENTS_DEVICE, "auto": _lib.RH_EVENTS_AUTO}[sink])
        compare(tab, model, orc, columns=False)
        live = np.arange(n)
        d = random_deltas(rng, model, live, n)   # matchIndex, flushIndex and follower commitIndex
        tab.push(d)
        model.apply(d)
        expect_w = model.watch(orc)
        expect = model.commit_batch(orc)
        assert expect[0].size > 1000 and expect[2].size > 1000 and expect_w[0].size > 100_000
        adv = expect[0]
        w = groups.make_deltas(adv, np.full(adv.size, _lib.RH_COL_COMMITTED), np.full(adv.size, 1 << 50),
                               np.full(adv.size, _lib.RH_OP_SET))
        stable, joint = conf_word(0b1111), conf_word(0b110011, old_mask=0b1111)
        victims = [int(s) for s in adv[:64]]
        tab.watch_async()                        # its record gather holds the side stream
        tk = tab.commit_async(watch_all=True)    # this one's gather queues behind it
        tab.push(w)                              # every column that gather reads, rewritten now
        for s in victims[:32]:
            tab.stop(s)
        for s in victims[:32]:
            tab.start(s, stable, 5_000, 4_000, 3_000)
        moved = [s for s in victims[32:] if model.conf[s] == stable]
        for s in moved:
            tab.reconf(s, joint, [0, 1, 2, 3, -1, -1])
        tk2 = tab.commit_async(watch_all=True)
        got = tab.commit_wait(tk)
        assert np.array_equal(got.advanced_slots, expect[0]) and np.array_equal(got.advanced_commit, expect[1])
        assert np.array_equal(got.watch_all_slots, expect[2]) and np.array_equal(got.watch_all_min, expect[3])
        levels = tab.watch_wait()   # its records are rebuilt from the level columns the restarts reset
        assert np.array_equal(levels["slot"], expect_w[0])
        assert np.array_equal(levels["min"], expect_w[1][0]) and np.array_equal(levels["majority"], expect_w[1][1])
        assert np.array_equal(levels["max"], expect_w[1][2]) and np.array_equal(levels["valid"] != 0, expect_w[2])
        # the model replays the same calls after the first evaluation
        model.apply(w)
        for s in victims[:32]:
            model.stop(s)
        for s in victims[:32]:
            model.start(s, stable, 5_000, 4_000, 3_000)
        for s in moved:
            model.reconf(s, joint, [0, 1, 2, 3, -1, -1])
        expect2 = model.commit_batch(orc)
        got2 = tab.commit_wait(tk2)
        assert np.array_equal(got2.advanced_slots, expect2[0]) and np.array_equal(got2.advanced_commit, expect2[1])
        assert np.array_equal(got2.watch_all_slots, expect2[2]) and np.array_equal(got2.watch_all_min, expect2[3])
    finally:
        tab.close()
