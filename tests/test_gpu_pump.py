"""The Java module's pump sequence (HipLeaderBookkeeper.tick) replayed in Python over a 2-shard
rh_node (ratis_amd.groups.LeaderPump), with divisions that apply the callbacks the way the
seams patch's LeaderStateImpl does (updateFromHip: updateCommit's follow-up and
watchRequests.update(ALL, min); commitIndexChanged's ALL_COMMITTED / MAJORITY_COMMITTED / MAJORITY;
WatchRequests queues only move forward, WatchRequests.java:146-149).  Checked against
tests/table_model.py step by step; in particular a step that carries ONLY follower commitIndex
reports (LeaderStateImpl.onFollowerCommitIndex -> commitIndexChanged, :606-622) must move the
ALL_COMMITTED / MAJORITY_COMMITTED levels with no commit event."""
import numpy as np
import pytest

from tests.table_model import COL_FLUSH, TableModel
from tests.test_gpu_table import conf_word

pytestmark = pytest.mark.gpu
IMIN = np.iinfo(np.int64).min


class Division:
    """The per-division state the seams touch: the commit index and the WatchRequests levels."""

    def __init__(self, commit):
        self.commit = commit
        self.levels = {"ALL": IMIN, "ALL_COMMITTED": IMIN, "MAJORITY_COMMITTED": IMIN, "MAJORITY": IMIN}
        self.notified = 0

    def _update(self, level, v):   # WatchRequests.update: a queue only moves forward
        self.levels[level] = max(self.levels[level], v)

    def on_commit(self, v):
        self.commit = max(self.commit, v)

    def on_watch_all(self, v):
        self._update("ALL", v)

    def on_watch_levels(self, mn, mj, mx):
        self._update("ALL_COMMITTED", mn)
        self._update("MAJORITY_COMMITTED", mj)
        self._update("MAJORITY", mx)
        self.notified += 1


def test_pump_replica_follower_commit_only_step(ctx, orc):
    from ratis_amd import groups
    rng = np.random.default_rng(61)
    cap, n = 500, 700
    with groups.RaftNode(0, cap, devices=[0, 0]) as node:
        pump = groups.LeaderPump(node)
        model = TableModel(2 * cap)
        slots = np.concatenate([np.arange(0, n // 2), cap + np.arange(0, n - n // 2)])
        divs = {}
        w = conf_word(0b1111)
        for s in slots:
            base = int(rng.integers(1 << 20, 1 << 30))
            node.start(int(s), w, base, base - 100, base - 500)
            model.start(int(s), w, base, base - 100, base - 500)
            divs[int(s)] = Division(base - 100)
            pump.register(int(s), divs[int(s)])
        want_levels = {int(s): {"ALL": IMIN, "ALL_COMMITTED": IMIN, "MAJORITY_COMMITTED": IMIN, "MAJORITY": IMIN}
                       for s in slots}

        def step(d):
            pump.emit(d)
            model.apply(d)
            got = pump.tick()
            a_s, a_c, w_s, w_m = model.commit_batch(orc)
            for s, v in zip(a_s, a_c):
                assert divs[int(s)].commit == v
            for s, v in zip(w_s, w_m):
                want_levels[int(s)]["ALL"] = max(want_levels[int(s)]["ALL"], int(v))
            m_s, m_lev, m_valid = model.watch(orc)
            for j, s in enumerate(m_s):
                if m_valid[j]:
                    for name, k in (("ALL_COMMITTED", 0), ("MAJORITY_COMMITTED", 1), ("MAJORITY", 2)):
                        want_levels[int(s)][name] = max(want_levels[int(s)][name], int(m_lev[k, j]))
            for s in slots:
                assert divs[int(s)].levels == want_levels[int(s)], int(s)
            assert got["commit"] == a_s.size
            return got

        # replies: matchIndex advances and flush advances -> commits, then the levels follow
        d = groups.make_deltas(np.repeat(slots, 5), np.tile([0, 1, 2, 3, COL_FLUSH], slots.size),
                               np.repeat(model.flush[slots], 5) + rng.integers(0, 300, 5 * slots.size))
        first = step(d)
        assert first["commit"] > n // 2 and first["watch_all"] > n // 2
        # follower commitIndex reports ONLY (LeaderStateImpl.onFollowerCommitIndex): no commit event,
        # but the ALL_COMMITTED / MAJORITY_COMMITTED levels move
        before = {int(s): dict(divs[int(s)].levels) for s in slots}
        cols = np.tile(16 + np.arange(4), slots.size)
        vals = np.repeat(model.commit[slots], 4) - rng.integers(0, 3, 4 * slots.size)
        got = step(groups.make_deltas(np.repeat(slots, 4), cols, vals))
        assert got["commit"] == 0 and got["watch_all"] == 0 and got["watch_levels"] > n // 2
        moved_ac = sum(divs[int(s)].levels["ALL_COMMITTED"] > before[int(s)]["ALL_COMMITTED"] for s in slots)
        moved_mc = sum(divs[int(s)].levels["MAJORITY_COMMITTED"] > before[int(s)]["MAJORITY_COMMITTED"] for s in slots)
        assert moved_ac > n // 2 and moved_mc > n // 2
        # and a quiet tick reports nothing
        got = step(groups.make_deltas(np.zeros(0, np.int64), 0, 0))
        assert got == {"commit": 0, "watch_all": 0, "watch_levels": 0}


def test_pump_replica_fallback_at_fifteen_followers(ctx, orc):
    """HipLeaderBookkeeper's FALLBACK in the pump replica: a division reconfigured to a joint
    change of two 8-peer confs needs 15 follower slots; its 15th addFollower makes it leave the
    table (slot stopped, counted, on_fallback called), after which its deltas are dropped and no
    event reaches it -- while a 6-follower division on the same node keeps exact parity with the
    model, tick after tick."""
    from ratis_amd import groups
    rng = np.random.default_rng(15)
    cap = 64
    with groups.RaftNode(0, cap, devices=[0, 0]) as node:
        pump = groups.LeaderPump(node)
        model = TableModel(2 * cap)
        fell = []

        class Cb(Division):
            def on_fallback(self):
                fell.append(True)

        a_cb, b_cb = Division(0), Cb(0)
        a = pump.division(3, a_cb)                 # shard 0
        b = pump.division(cap + 5, b_cb)           # shard 1
        a_peers = [f"a{i}" for i in range(6)]
        b_old = [f"b{i}" for i in range(8)]
        b_new = ["b0"] + [f"c{i}" for i in range(7)]   # union with b_old: 15 followers
        for p in a_peers:
            a.add_follower(p)
        for p in b_old:
            b.add_follower(p)
        wa, wb = a.conf_word(a_peers), b.conf_word(b_old)
        a.start(wa, 10_000, 9_000, 9_500)
        b.start(wb, 20_000, 19_000, 19_500)
        model.start(3, wa, 10_000, 9_000, 9_500)
        model.start(cap + 5, wb, 20_000, 19_000, 19_500)
        assert node.tables[0].tier_width(3) == 6 and node.tables[1].tier_width(5) == 8

        def step(deltas_a, deltas_b):
            for k, v in deltas_a:
                a.match_index(k, v)
            for k, v in deltas_b:
                b.match_index(k, v)
            for k, v in deltas_a:
                model.apply(groups.make_deltas([3], [k], [v]))
            if not b.fallback:
                for k, v in deltas_b:
                    model.apply(groups.make_deltas([cap + 5], [k], [v]))
            before_b = b_cb.commit
            got = pump.tick()
            a_s, a_c, _, _ = model.commit_batch(orc)
            model.watch(orc)
            if 3 in a_s.tolist():
                assert a_cb.commit == int(a_c[a_s.tolist().index(3)])
            return got, before_b

        step([(k, 10_000 + 50 * k) for k in range(6)], [(k, 20_000 + 10 * k) for k in range(8)])
        assert a_cb.commit > 9_000 and b_cb.commit > 19_000
        # the joint change: new peers get slots 8..13, the 15th peer has none -> fallback
        slots = [b.add_follower(p) for p in b_new]
        assert slots == [0] + list(range(8, 14)) + [-1]
        assert b.fallback and fell == [True] and pump.fallbacks == {"FOLLOWER_SLOTS": 1}
        assert node.tables[1].tier_width(5) == 0           # the slot left the table
        b.reconf(b.conf_word(b_new, b_old))                # ignored: the division runs in Java now
        model.stop(cap + 5)
        a.flush_index(20_000)                              # the leader's log grows: commits can move on
        model.apply(groups.make_deltas([3], [COL_FLUSH], [20_000]))
        for t in range(4):
            _, before_b = step([(k, 10_500 + 100 * t + int(rng.integers(0, 90))) for k in range(6)],
                               [(k, 30_000 + t) for k in range(8)])
            assert b_cb.commit == before_b                 # no event reaches the fallen-back division
        assert a_cb.commit >= 10_500


def test_pump_replica_recycled_slot_after_stale_delta_in_another_buffer(ctx, orc):
    """a stale MAX(matchIndex) of a removed peer sits in one producer thread's buffer
    when another thread recycles the peer's slot for a new follower.  The new follower must start
    at -1 (FollowerInfoImpl.java:42-43) whatever order the buffers are pushed in: the reset is
    pushed after every buffer (PumpDivision._reset_slot / HipLeaderBookkeeper.resetFollowerSlot),
    so the commit does not advance on the old peer's index."""
    import threading

    from ratis_amd import _lib, groups
    cap = 16
    with groups.RaftNode(0, cap, devices=[0]) as node:
        pump = groups.LeaderPump(node)
        cb = Division(0)
        d = pump.division(2, cb)
        peers = ["p0", "p1", "p2", "p3"]
        for p in peers:
            d.add_follower(p)
        d.start(d.conf_word(peers), 5_000, 1_000, 1_000)
        for k in range(4):                       # every follower at 1_500: commit 1_500
            d.match_index(k, 1_500)
        pump.tick()
        assert cb.commit == 1_500
        # thread B's buffer is registered (pushed) BEFORE thread A's; A buffers a stale high
        # matchIndex for p3's slot, then B removes p3 and gives the slot to p4 -- the order in which
        # a plain drain would push B's reset SETs ahead of A's stale MAX
        import queue
        jobs = queue.Queue()

        def worker():
            while True:
                f = jobs.get()
                if f is None:
                    return
                f()
                jobs.task_done()
        tb = threading.Thread(target=worker)
        tb.start()
        jobs.put(lambda: d.flush_index(5_000))      # B's first delta: B's buffer registered first
        jobs.join()
        t_old = threading.Thread(target=lambda: d.match_index(3, 4_000))   # A: the stale MAX
        t_old.start()
        t_old.join()

        def recycle():
            d.remove_follower("p3")
            assert d.add_follower("p4") == 3
        jobs.put(recycle)
        jobs.join()
        jobs.put(None)
        tb.join()
        for k in range(3):                       # the three old followers reach 4_000
            d.match_index(k, 4_000)
        pump.tick()
        got = node.tables[0].read(_lib.rh_col_match(3), 2, 1)
        assert int(got[0]) == -1                 # the new follower's matchIndex, not the stale 4_000
        # conf {self, p0, p1, p2, p4}: the majority (3 of 5) is at 4_000 -- the commit moves there
        # only because three OLD followers reached it, never by p4's inherited value
        assert cb.commit == 4_000
