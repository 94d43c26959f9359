"""The exact sequences the reference's own unit tests assert for the commit side, replayed through
the oracle (CPU) and through the C ABI on the GPU.  Fixture: tests/golden/reference_sequences.json
(tests/golden/make_golden.py transcribes it from TestRaftLogIndex.java:44-83 and
TestPeerConfiguration.java:45-70).

  * RaftLogIndex.updateToMax / setUnconditionally sequences -> rh_push_deltas RH_OP_MAX / RH_OP_SET
    on the columns FollowerInfoImpl drives with them (matchIndex, FollowerInfoImpl.java:93-95,
    147-151; follower commitIndex :103-105), read back after every step;
  * PeerConfiguration.hasMajority / majorityRejectVotes (odd and even quorums) -> conf words through
    rh_commit_soa_launch: a voter set reaches the majority index iff it is a majority, the same
    `num > size / 2` rule the kernel's sorted[(n - 1) / 2] must agree with."""
import json
import os

import numpy as np
import pytest

from tests.table_model import OP_MAX, OP_SET, TableModel

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = json.load(open(os.path.join(HERE, "golden", "reference_sequences.json")))
OPS = {"updateToMax": OP_MAX, "setUnconditionally": OP_SET}
HI, LO = 100, 10
ACTIVE, SELF = 1 << 31, 1 << 14


def _table_sections():
    return [s for s in FIX["raft_log_index"] if s["method"] in OPS]


def _peer_rows():
    """One commit row per assertion: followers = the voters other than self (slots 0..), matchIndex
    HI for the peers that count (others / non-rejecting), LO for the rest; self = flushIndex HI.
    The row's commit reaches HI iff the counting set is a majority of the conf."""
    rows = []
    for c in FIX["peer_configuration"]:
        followers = [p for p in c["voters"] if p != c["self"]]
        for h in c["has_majority"]:
            rows.append((c["name"], [HI if p in h["others"] else LO for p in followers], h["expected"]))
        for r in c["majority_reject_votes"]:   # rejected peers lag: a majority remains iff not rejected
            rows.append((c["name"], [LO if p in r["rejected"] else HI for p in followers], not r["expected"]))
    return rows


def _peer_arrays():
    rows = _peer_rows()
    n, F = len(rows), 3
    follower = np.full((F, n), -1, dtype=np.int64)
    conf = np.zeros(n, dtype=np.uint32)
    for i, (_, v, _) in enumerate(rows):
        follower[: len(v), i] = v
        conf[i] = ((1 << len(v)) - 1) | SELF | ACTIVE
    flush = np.full(n, HI, dtype=np.int64)
    commit = np.zeros(n, dtype=np.int64)
    ts = np.zeros(n, dtype=np.int64)
    want = np.array([HI if e else LO for _, _, e in rows], dtype=np.int64)
    return follower, flush, conf, commit, ts, want


def test_fixture_covers_the_reference_tests():
    kinds = [s["method"] for s in FIX["raft_log_index"]]
    assert kinds == ["updateIncreasingly", "updateToMax", "setUnconditionally", "updateUnconditionally"]
    assert [c["name"] for c in FIX["peer_configuration"]] == ["testOddNodesQuorum", "testEvenNodeQuorum"]
    assert len(_peer_rows()) == 6


def test_raft_log_index_sequences_on_the_table_model():
    for s in _table_sections():
        m = TableModel(1)
        m.start(0, ACTIVE | 0b11, 0, 0, 0)
        m._apply_one(0, 0, OP_SET, s["initial"])          # new RaftLogIndex(name, initialValue)
        for st in s["steps"]:
            m._apply_one(0, 0, OPS[s["method"]], st["arg"])
            assert m.match[0, 0] == st["after"], (s["method"], st)


def test_peer_configuration_quorums_on_the_oracle(orc):
    follower, flush, conf, commit, ts, want = _peer_arrays()
    ref = orc.commit_soa(follower, flush, conf, mode=0, gap=-1, commit_in=commit, term_start=ts)
    assert np.array_equal(ref["commit"], want)


@pytest.mark.gpu
@pytest.mark.parametrize("column", [0, 5, 16, 21])   # matchIndex / follower commitIndex of slots 0, 5
def test_raft_log_index_sequences_on_gpu(ctx, column):
    from ratis_amd import groups
    with groups.RaftGroupTable(ctx, capacity=8) as tab:
        for slot, s in enumerate(_table_sections()):
            tab.start(slot, ACTIVE | SELF | 0b111111, 1000, 0, 0)
            tab.push(groups.make_deltas([slot], [column], [s["initial"]], [OP_SET]))
            for st in s["steps"]:                          # one step per push, read back after each
                tab.push(groups.make_deltas([slot], [column], [st["arg"]], [OPS[s["method"]]]))
                assert tab.read(column)[slot] == st["after"], (s["method"], st)
            # the whole sequence in ONE push: the library cuts it so the order is kept
            tab.push(groups.make_deltas([slot] * (1 + len(s["steps"])), [column] * (1 + len(s["steps"])),
                                        [s["initial"]] + [st["arg"] for st in s["steps"]],
                                        [OP_SET] + [OPS[s["method"]]] * len(s["steps"])))
            assert tab.read(column)[slot] == s["steps"][-1]["after"], s["method"]


@pytest.mark.gpu
def test_peer_configuration_quorums_on_gpu(ctx):
    from tests.test_gpu_commit import _run_gpu
    follower, flush, conf, commit, ts, want = _peer_arrays()
    got = _run_gpu(ctx, follower, flush, conf, commit, ts, mode=0, gap=-1)
    assert np.array_equal(got["commit"], want), (got["commit"], want)
