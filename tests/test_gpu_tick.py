"""GPU parity of rh_tick_async, the pump tick's two evaluations in one call (round 6): updateCommit
of the rows marked since the last evaluation, then commitIndexChanged of every row whose levels may
have moved (LeaderStateImpl.java:946-950, then 612-622, per division).  When both kinds' dirty rows
are listed the library runs them in ONE launch (table_tick_kernel: a row's commitIndexChanged in the
lane that just evaluated its updateCommit, the watch list's other rows after, each claimed exactly once
by an atomic on its watch flag); otherwise it falls back to the two launches.  Checked

  * against tests/table_model.py (the reference's semantics over the oracle's arithmetic) through
    random lifecycles over every tier width -- control ops between ticks (the fallback), sparse ticks
    (the fused launch), ticks past the list capacity (the tile fallback), SET deltas, the gap clamp;
  * against a twin table driven by the two calls (commit_async + watch_async), for every event sink
    and with / without watch-ALL: every list and the table's columns identical, on a table of 300k
    rows (the fused launch spread over every region of both lists)."""
import numpy as np
import pytest

from tests.table_model import TableModel
from tests.test_gpu_table import COL_COMMITTED, COL_FLUSH, conf_word, random_deltas

pytestmark = pytest.mark.gpu


def _tick(tab, watch_all=True):
    tk = tab.tick_async(watch_all=watch_all)
    return tab.commit_wait(tk), tab.watch_wait()


def _expect(got, ev, model, orc):
    a_s, a_c, w_s, w_m = model.commit_batch(orc)
    assert np.array_equal(got.advanced_slots, a_s)
    assert np.array_equal(got.advanced_commit, a_c)
    assert np.array_equal(got.watch_all_slots, w_s)
    assert np.array_equal(got.watch_all_min, w_m)
    m_s, m_lev, m_valid = model.watch(orc)
    assert np.array_equal(ev["slot"].astype(np.int64), m_s)
    assert np.array_equal(ev["min"], m_lev[0]) and np.array_equal(ev["majority"], m_lev[1])
    assert np.array_equal(ev["max"], m_lev[2]) and np.array_equal(ev["valid"].astype(bool), m_valid)
    return a_s.size + w_s.size + m_s.size


@pytest.mark.parametrize("seed", [31, 32])
def test_tick_matches_model_every_width(ctx, orc, seed):
    from ratis_amd import groups
    rng = np.random.default_rng(seed)
    n, gap = 40_000, 300
    model = TableModel(n, gap=gap)

    def rand_conf():
        F = int(rng.integers(1, 15))
        new = int(rng.integers(1, 1 << F))
        if rng.random() < 0.3:
            return conf_word(new, old_mask=int(rng.integers(0, 1 << F)), self_new=rng.random() < 0.9,
                             self_old=rng.random() < 0.9)
        return conf_word(new, self_new=rng.random() < 0.95)

    with groups.RaftGroupTable(ctx, capacity=n, gap_threshold=gap) as tab:
        tab.set_timing(True)
        for s in range(0, n, 3):   # a third of the slots started, over every width
            b = int(rng.integers(1000, 1 << 40))
            args = (s, rand_conf(), b, b - int(rng.integers(0, 2000)), b - int(rng.integers(-500, 3000)))
            tab.start(*args)
            model.start(*args)
        fused = fallback = events = 0
        for step in range(40):
            if step % 8 == 7:   # control ops: the lists are dropped, this tick runs the two launches
                for s in rng.choice(n, size=60, replace=False):
                    s = int(s)
                    r = rng.random()
                    if not model.started[s] or r < 0.3:
                        b = int(rng.integers(1000, 1 << 40))
                        args = (s, rand_conf(), b, b - int(rng.integers(0, 2000)), b - int(rng.integers(-500, 3000)))
                        tab.start(*args)
                        model.start(*args)
                    elif r < 0.8:
                        c = rand_conf()
                        src = [int(x) for x in rng.integers(-1, 14, size=14)]
                        tab.reconf(s, c, src)
                        model.reconf(s, c, src)
                    else:
                        tab.stop(s)
                        model.stop(s)
            live = np.nonzero(model.started)[0]
            k = int(rng.choice([0, 3, 64, 400, 1100, 6000]))   # 6000: past the lists (1250 marks)
            d = random_deltas(rng, model, live, k, set_frac=0.05 if step % 3 == 0 else 0.0)
            tab.push(d)
            model.apply(d)
            got, ev = _tick(tab)
            events += _expect(got, ev, model, orc)
            sp = tab.last_timing_split()
            if sp["fused"]:
                fused += 1
                assert sp["eval_ms"] > 0 and sp["gather_ms"] == 0
            else:
                fallback += 1
            if step % 10 == 9:
                for col in [0, 3, 13, 16, 29, COL_FLUSH, COL_COMMITTED, 34, 35]:
                    assert np.array_equal(tab.read(col), model.column(col)), col
        # both forms ran and the comparisons were not vacuous
        assert fused >= 15 and fallback >= 5, (fused, fallback)
        assert events > 1000, events
        # nothing marked: the fused launch over empty lists reports nothing
        got, ev = _tick(tab)
        assert got.advanced_slots.size == 0 and got.watch_all_slots.size == 0 and ev.size == 0
        assert tab.last_timing_split()["fused"]


def _snapshot_table(ctx, n, seed, sink):
    from ratis_amd import _lib, groups, workload
    tiers = workload.commit_snapshot(n, joint_frac=0.1, peers=5, seed=seed)
    tab = groups.RaftGroupTable(ctx, capacity=sum(t.n for t in tiers))
    tab.set_event_sink({"device": _lib.RH_EVENTS_DEVICE, "host_mapped": _lib.RH_EVENTS_HOST_MAPPED,
                        "auto": _lib.RH_EVENTS_AUTO}[sink])
    first = 0
    for h in tiers:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        first += h.n
    return tab, tiers, first


@pytest.mark.parametrize("sink,watch_all", [("auto", True), ("host_mapped", False), ("device", True)])
def test_tick_matches_two_calls(ctx, sink, watch_all):
    """The same replies into two tables, one ticked by rh_tick_async, one by the two calls: every
    list identical (as sets: the fused launch lists in its own order) and the columns identical."""
    from ratis_amd import groups
    n = 300_000
    a, tiers, n = _snapshot_table(ctx, n, 77, sink)
    b, _, _ = _snapshot_table(ctx, n, 77, sink)
    a.set_timing(True)
    rng = np.random.default_rng(78)
    match = np.concatenate([h.follower[:4] for h in tiers], axis=1)
    try:
        fused = 0
        for step in range(14):
            # 1.5 k deltas, each counted as a possible mark of both kinds: 30_000 goes past the lists (9375)
            k = [0, 40, 2000, 6000, 30_000, 6000, 512][step % 7]
            both = rng.choice(n, size=k // 2, replace=False)
            col = rng.integers(0, 4, size=both.size)
            match[col, both] += rng.integers(1, 300, size=both.size)
            # replies (matchIndex + commitIndex of one follower), plus commitIndex-only deltas on other
            # rows (watch list only) and matchIndex-only deltas (commit list only)
            wonly = rng.choice(n, size=k // 4, replace=False)
            conly = rng.choice(n, size=k // 4, replace=False)
            wc, cc = rng.integers(0, 4, size=wonly.size), rng.integers(0, 4, size=conly.size)
            match[cc, conly] += rng.integers(0, 50, size=conly.size)
            d = groups.make_deltas(np.concatenate([both, both, wonly, conly]),
                                   np.concatenate([col, 16 + col, 16 + wc, cc]),
                                   np.concatenate([match[col, both], match[col, both] - rng.integers(0, 3, both.size),
                                                   match[wc, wonly] - 1, match[cc, conly]]))
            a.push(d)
            b.push(d)
            ga, ea = _tick(a, watch_all)
            fused += a.last_timing_split()["fused"]
            tk = b.commit_async(watch_all=watch_all)
            b.watch_async()
            gb, eb = b.commit_wait(tk), b.watch_wait()
            assert np.array_equal(ga.advanced_slots, gb.advanced_slots)
            assert np.array_equal(ga.advanced_commit, gb.advanced_commit)
            assert np.array_equal(ga.watch_all_slots, gb.watch_all_slots)
            assert np.array_equal(ga.watch_all_min, gb.watch_all_min)
            assert np.array_equal(ea, eb)
            if k == 6000:
                assert ga.advanced_slots.size > 100 and ea.size > 100
            if step % 7 == 6:
                for c in [0, 3, 16, 19, COL_COMMITTED]:
                    assert np.array_equal(a.read(c), b.read(c)), c
        if sink == "device":
            assert fused == 0   # the DEVICE sink keeps the two launches
        else:
            assert fused >= 8, fused
    finally:
        a.close()
        b.close()


def test_tick_ticket_rotation_and_misuse(ctx, orc):
    """rh_tick_async's tickets rotate with rh_commit_batch_async's (three result sets): ticks issued
    back to back without waits are ordered, a superseded ticket fails, the watch list is the last
    tick's; a watch wait with none outstanding fails."""
    import ctypes

    from ratis_amd import _lib, groups, workload
    rng = np.random.default_rng(5)
    n = 20_000
    model = TableModel(n)
    tiers = workload.commit_snapshot(n, joint_frac=0.1, peers=5, seed=6)
    with groups.RaftGroupTable(ctx, capacity=sum(t.n for t in tiers)) as tab:
        first = 0
        for h in tiers:
            tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            model.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            first += h.n
        live = np.arange(first)
        _expect(*_tick(tab), model, orc)
        tickets = []
        for step in range(5):
            d = random_deltas(rng, model, live, 300)
            tab.push(d)
            model.apply(d)
            tickets.append(tab.tick_async(watch_all=True))
            expect = model.commit_batch(orc)
            wexp = model.watch(orc)
        for tk in tickets[:-3]:
            with pytest.raises(_lib.RatisHipError):
                tab.commit_wait(tk)
        got = tab.commit_wait(tickets[-1])
        assert np.array_equal(got.advanced_slots, expect[0]) and np.array_equal(got.advanced_commit, expect[1])
        ev = tab.watch_wait()
        assert np.array_equal(ev["slot"].astype(np.int64), wexp[0])
        assert np.array_equal(ev["min"], wexp[1][0]) and np.array_equal(ev["max"], wexp[1][2])
        with pytest.raises(_lib.RatisHipError):
            tab.watch_wait()
        assert tab._lib.rh_tick_async(tab.handle, 0, None) != 0   # NULL ticket
        tk = ctypes.c_uint64()
        assert tab._lib.rh_tick_async(tab.handle, 8, ctypes.byref(tk)) != 0   # unknown flag


def test_tick_with_concurrent_producers(ctx, orc):
    """4 producer threads push reply deltas (matchIndex, follower commitIndex, flushIndex MAXes) in
    small calls while the main thread ticks (rh_tick_async + both waits) as fast as it can: no tick
    reports a slot twice in one list, and after the producers are done and a last tick, every slot's
    last reported commit index and levels -- and the table's columns -- are the model's for the whole
    delta set (MAX deltas commute; commit and levels only rise)."""
    import threading
    import time

    from ratis_amd import groups, workload
    rng = np.random.default_rng(808)
    n = 50_000
    model = TableModel(n)
    tiers = workload.commit_snapshot(n, joint_frac=0.1, peers=5, seed=81)
    tab = None
    try:
        tab = groups.RaftGroupTable(ctx, capacity=sum(t.n for t in tiers))
        first = 0
        for h in tiers:
            tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            model.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            first += h.n
        _expect(*_tick(tab), model, orc)
        live = np.arange(first)
        T = 4
        work = []
        for t in range(T):
            chunks = []
            for _ in range(60):
                k = int(rng.integers(1, 300))
                d = random_deltas(rng, model, live, k)   # MAX only: match, follower commitIndex, flush
                chunks.append(d)
            work.append(chunks)
        errors = []

        def producer(t):
            try:
                for d in work[t]:
                    tab.push(d)
                    time.sleep(1e-4)   # replies trickle in across many ticks
            except Exception as e:  # noqa: BLE001
                errors.append(e)

        th = [threading.Thread(target=producer, args=(t,)) for t in range(T)]
        for x in th:
            x.start()
        last_commit, last_levels, ticks = {}, {}, 0

        def collect(got, ev):
            assert np.unique(got.advanced_slots).size == got.advanced_slots.size
            assert np.unique(ev["slot"]).size == ev.size
            for s_, v in zip(got.advanced_slots.tolist(), got.advanced_commit.tolist()):
                last_commit[s_] = v
            for e in ev:
                last_levels[int(e["slot"])] = (int(e["min"]), int(e["majority"]), int(e["max"]), bool(e["valid"]))

        while any(x.is_alive() for x in th):
            collect(*_tick(tab))
            ticks += 1
        for x in th:
            x.join()
        assert not errors, errors
        collect(*_tick(tab))
        for t in range(T):
            for d in work[t]:
                model.apply(d)
        a_s, a_c, _, _ = model.commit_batch(orc)
        m_s, m_lev, m_valid = model.watch(orc)
        assert {s_: last_commit[s_] for s_ in a_s.tolist()} == dict(zip(a_s.tolist(), a_c.tolist()))
        assert set(last_commit) == set(a_s.tolist())
        want = {int(s_): (int(m_lev[0][i]), int(m_lev[1][i]), int(m_lev[2][i]), bool(m_valid[i]))
                for i, s_ in enumerate(m_s.tolist())}
        assert last_levels == want
        for col in [0, 3, 16, 19, COL_FLUSH, COL_COMMITTED]:
            assert np.array_equal(tab.read(col), model.column(col)), col
        assert ticks >= 10 and len(last_commit) > 100 and len(last_levels) > 100, (ticks, len(last_commit))
    finally:
        if tab is not None:
            tab.close()
