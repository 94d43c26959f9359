"""Watch-level, joint-consensus and leader-lease scenarios transcribed from the reference's own
integration tests (tests/golden/reference_scenarios.json: WatchRequestTests.java:221-371 and
LeaderElectionTests.java:725-795, each step citing the test lines it restates), replayed on three
backends that must all reach the test's verdicts:

  literal  the oracle's restatements evaluated on the literal per-peer state after every step
           (orc_commit_soa for updateCommit / commitIndexChanged, orc_lease_soa for hasLease);
  model    tests/table_model.py, the resident table's host model (event semantics: only changed
           results are reported), with the lease state beside it;
  gpu      rh_node on the GPU (-m gpu), driven the way the Java module drives it: the conf word of
           the division's follower slots, deltas per reply, rh_node_commit_batch /
           rh_node_watch_levels / rh_node_lease_batch.

A watch at log index L at level X counts as done when the last level reported for X is >= L
(WatchRequests.update)."""
import json
import os

import numpy as np
import pytest

from tests.table_model import IMIN, TableModel

HERE = os.path.dirname(os.path.abspath(__file__))
SC = json.load(open(os.path.join(HERE, "golden", "reference_scenarios.json")))["scenarios"]
PEERS = {"f0": 0, "f1": 1, "n0": 2, "n1": 3}
F = 4
T0 = 1 << 40      # System.nanoTime() origin of the lease scenarios
MS = 1_000_000
LEVELS = ("ALL", "ALL_COMMITTED", "MAJORITY_COMMITTED", "MAJORITY")
COL_FLUSH, OP_MAX, OP_SET = 32, 0, 1


def conf_word(new, old=None, self_new=True, self_old=True):
    w = sum(1 << PEERS[p] for p in new) | (1 << 14 if self_new else 0) | (1 << 31)
    if old is not None:
        w |= (1 << 15) | (sum(1 << PEERS[p] for p in old) << 16) | ((1 << 30) if self_old else 0)
    return w & 0xFFFFFFFF


def width_of(conf):
    m = (conf & 0x3FFF) | ((conf >> 16) & 0x3FFF)
    w = m.bit_length()
    return 2 if w <= 2 else 2 * ((w + 1) // 2)


class Literal:
    """The reference's per-division state, literally: FollowerInfo indices and timestamps per
    follower slot, the leader's indices, the LeaderLease; verdicts from the oracle."""

    def __init__(self, orc):
        self.orc = orc
        self.levels = {k: IMIN for k in LEVELS}

    def start(self, conf, flush, commit, tstart):
        self.conf, self.flush, self.commit, self.tstart = conf, flush, commit, tstart
        self.width = width_of(conf)
        self.match = np.full(F, -1, np.int64)
        self.fcommit = np.full(F, -1, np.int64)
        self.ts = np.full(F, IMIN, np.int64)
        self.lease, self.lease_on = IMIN, 0
        self.levels = {k: IMIN for k in LEVELS}

    def stop(self):
        pass

    def reconf(self, conf):
        w = width_of(conf)
        for k in range(self.width, w):   # a wider tier's new follower slots start as new FollowerInfos
            self.match[k], self.fcommit[k], self.ts[k] = -1, -1, IMIN
        self.conf, self.width = conf, w

    def delta(self, k, col, op, v):
        arr = {"match": self.match, "fcommit": self.fcommit, "ts": self.ts}[col]
        if k < self.width:
            arr[k] = v if op == OP_SET else max(arr[k], v)

    def set_flush(self, v):
        self.flush = max(self.flush, v)

    def lease_start(self, now, enabled):
        self.lease, self.lease_on = now, int(enabled)
        self.ts[: self.width] = now

    def evaluate(self):
        w = np.array([self.conf], np.uint32)
        r = self.orc.commit_soa(self.match.reshape(F, 1), np.array([self.flush]), w, mode=0, gap=-1,
                                commit_in=np.array([self.commit]), term_start=np.array([self.tstart]))
        if r["valid_bits"][0] & 1:
            self.commit = int(r["commit"][0])
            self.levels["ALL"] = int(r["min"][0])
        r = self.orc.commit_soa(self.fcommit.reshape(F, 1), np.array([self.commit]), w, mode=1, gap=-1,
                                commit_in=np.array([self.commit]), term_start=np.array([self.tstart]))
        if r["valid_bits"][0] & 1:
            self.levels["ALL_COMMITTED"], self.levels["MAJORITY_COMMITTED"], self.levels["MAJORITY"] = (
                int(r["min"][0]), int(r["maj"][0]), int(r["max"][0]))
        return self.commit, dict(self.levels)

    def has_lease(self, now, timeout_ms):
        en = np.array([self.lease_on], np.uint64)
        r = self.orc.lease_soa(self.ts.reshape(F, 1), np.array([self.conf], np.uint32), np.array([self.lease]), now,
                               timeout_ms, enabled_bits=en)
        self.lease = int(r["lease"][0])
        return bool(r["has_lease_bits"][0] & 1)


class Model(Literal):
    """tests/table_model.py (slot 3 of a small table) with its event semantics; the lease state as
    the table keeps it (timestamp / lease / enabled columns), hasLease by the oracle."""

    SLOT = 3

    def __init__(self, orc):
        super().__init__(orc)
        self.tm = TableModel(8)

    def start(self, conf, flush, commit, tstart):
        super().start(conf, flush, commit, tstart)
        self.tm.start(self.SLOT, conf, flush, commit, tstart)

    def stop(self):
        self.tm.stop(self.SLOT)

    def reconf(self, conf):
        super().reconf(conf)
        self.tm.reconf(self.SLOT, conf)

    def delta(self, k, col, op, v):
        super().delta(k, col, op, v)
        if col != "ts" and k < self.width:
            from ratis_amd.groups import make_deltas
            self.tm.apply(make_deltas([self.SLOT], [k if col == "match" else 16 + k], [v], [op]))

    def set_flush(self, v):
        super().set_flush(v)
        from ratis_amd.groups import make_deltas
        self.tm.apply(make_deltas([self.SLOT], [COL_FLUSH], [v], [OP_MAX]))

    def evaluate(self):
        _, _, w_s, w_m = self.tm.commit_batch(self.orc)
        for s, m in zip(w_s, w_m):
            if s == self.SLOT and m != IMIN:
                self.levels["ALL"] = int(m)
        m_s, m_lev, m_valid = self.tm.watch(self.orc)
        for i, s in enumerate(m_s):
            if s == self.SLOT and m_valid[i]:
                self.levels["ALL_COMMITTED"], self.levels["MAJORITY_COMMITTED"], self.levels["MAJORITY"] = (
                    int(m_lev[0, i]), int(m_lev[1, i]), int(m_lev[2, i]))
        return int(self.tm.commit[self.SLOT]), dict(self.levels)


class Gpu:
    """rh_node on the GPU, as the Java module drives it (node slot 5 of shard 0)."""

    SLOT = 5

    def __init__(self, orc):
        from ratis_amd import groups
        self.node = groups.RaftNode(0, 16, devices=[0])
        self.levels = {k: IMIN for k in LEVELS}
        self.width = 0

    def close(self):
        self.node.close()

    def _push(self, cols, vals, ops):
        from ratis_amd.groups import make_deltas
        self.node.push(make_deltas([self.SLOT] * len(cols), cols, vals, ops))

    def start(self, conf, flush, commit, tstart):
        self.node.start(self.SLOT, conf, flush, commit, tstart)
        self.width = width_of(conf)
        self.levels = {k: IMIN for k in LEVELS}

    def stop(self):
        self.node.stop(self.SLOT)

    def reconf(self, conf):
        self.node.reconf(self.SLOT, conf)
        self.width = width_of(conf)

    def delta(self, k, col, op, v):
        if k < self.width:   # HipLeaderBookkeeper.emit: only columns the division's tier has
            self._push([{"match": k, "fcommit": 16 + k, "ts": 48 + k}[col]], [v], [op])

    def set_flush(self, v):
        self._push([COL_FLUSH], [v], [OP_MAX])

    def lease_start(self, now, enabled):
        self.node.lease_start(self.SLOT, now, enabled)

    def evaluate(self):
        adv, wall = self.node.update_commit(16)
        for e in wall:
            if e["slot"] == self.SLOT and e["value"] != IMIN:
                self.levels["ALL"] = int(e["value"])
        for e in self.node.watch_levels(16):
            if e["slot"] == self.SLOT and e["valid"]:
                self.levels["ALL_COMMITTED"], self.levels["MAJORITY_COMMITTED"], self.levels["MAJORITY"] = (
                    int(e["min"]), int(e["majority"]), int(e["max"]))
        return int(self.node.tables[0].read(33)[self.SLOT]), dict(self.levels)

    def has_lease(self, now, timeout_ms):
        return bool(self.node.lease_batch(now, timeout_ms)[self.SLOT])


def replay(sc, b):
    """Runs one scenario on backend b; returns the verdicts (step index, what, value)."""
    out = []
    timeout = sc.get("timeout_ms", 75)
    for i, st in enumerate(sc["steps"]):
        op = st["op"]
        if op == "start":
            b.start(conf_word(st["new"], st.get("old")), st["flush"], st["commit"], st["term_start"])
        elif op == "stop":
            b.stop()
        elif op == "reconf":
            b.reconf(conf_word(st["new"], st.get("old")))
        elif op == "reply":
            k = PEERS[st["peer"]]
            if "sent_ms" in st:   # updateLastRespondedAppendEntriesSendTime (GrpcLogAppender.java:491)
                b.delta(k, "ts", OP_SET, T0 + st["sent_ms"] * MS)
            b.delta(k, "match", OP_MAX, st["match"])   # updateMatchIndex (:516)
        elif op == "follower_commit":
            b.delta(PEERS[st["peer"]], "fcommit", OP_MAX, st["value"])
        elif op == "flush":
            b.set_flush(st["value"])
        elif op == "lease_start":
            b.lease_start(T0 + st["now_ms"] * MS, st["enabled"])
        elif op == "add_follower":   # addFollower: a new FollowerInfo (-1, -1, lastRpcTime = now)
            k = PEERS[st["peer"]]
            b.delta(k, "match", OP_SET, -1)
            b.delta(k, "fcommit", OP_SET, -1)
            b.delta(k, "ts", OP_SET, T0 + st["now_ms"] * MS)
        elif op == "expect_commit":
            out.append((i, "commit", b.evaluate()[0]))
        elif op == "expect_watch":
            levels = b.evaluate()[1]
            out.append((i, "watch", {k: levels[k] >= st["index"] for k in LEVELS}))
        elif op == "expect_lease":
            b.evaluate()
            out.append((i, "lease", b.has_lease(T0 + st["now_ms"] * MS, timeout)))
        else:
            raise ValueError(op)
    return out


def expected(sc):
    out = []
    for i, st in enumerate(sc["steps"]):
        if st["op"] == "expect_commit":
            out.append((i, "commit", st["value"]))
        elif st["op"] == "expect_watch":
            out.append((i, "watch", {k: st[k] for k in LEVELS}))
        elif st["op"] == "expect_lease":
            out.append((i, "lease", st["value"]))
    return out


def test_fixture_cites_the_reference_tests():
    assert len(SC) == 4
    for sc in SC:
        assert "WatchRequestTests.java:" in sc["cites"] or "LeaderElectionTests.java:" in sc["cites"]
        assert any(st["op"].startswith("expect_") and "cite" in st for st in sc["steps"])


@pytest.mark.parametrize("sc", SC, ids=[s["name"] for s in SC])
def test_scenario_on_oracle(orc, sc):
    assert replay(sc, Literal(orc)) == expected(sc)


@pytest.mark.parametrize("sc", SC, ids=[s["name"] for s in SC])
def test_scenario_on_table_model(orc, sc):
    assert replay(sc, Model(orc)) == expected(sc)


@pytest.mark.gpu
@pytest.mark.parametrize("sc", SC, ids=[s["name"] for s in SC])
def test_scenario_on_gpu_node(ctx, orc, sc):
    b = Gpu(orc)
    try:
        assert replay(sc, b) == expected(sc)
    finally:
        b.close()
