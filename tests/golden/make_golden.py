"""Generates the committed golden fixtures under tests/golden/.  Run from the repo root:

    python tests/golden/make_golden.py

Sources of truth (the reference is pure Java and cannot run in this image):
  * crc_reference.json -- SHA-256 of the 2048-word slicing table parsed from the T[] literal
    of ratis-common/src/main/java/org/apache/ratis/util/PureJavaCrc32C.java:167-688 (read as
    text from /root/reference), plus RFC 3720 B.4 known answers.  Only the hash and the
    answers are stored, not the table text.
  * commit_cases.json -- hand-derived cases of LeaderStateImpl.getMajorityMin / updateCommit
    (LeaderStateImpl.java:904-1026) and RaftLogBase.updateCommitIndex (RaftLogBase.java:121-142);
    every expected value is written by hand below and re-checked here against both oracle
    restatements before it is saved.
  * reference_sequences.json -- the exact sequences two reference unit tests assert, transcribed
    with the values the test computes: TestRaftLogIndex.testIndex (TestRaftLogIndex.java:44-83:
    RaftLogIndex.updateIncreasingly / updateToMax / setUnconditionally / updateUnconditionally,
    each step's `updated` flag and the index after it) and TestPeerConfiguration's odd/even quorum
    cases (TestPeerConfiguration.java:45-70: hasMajority / majorityRejectVotes), re-checked here
    against a restatement of RaftLogIndex.java:45-86 and PeerConfiguration.java:157-184.
  * raftlog_rw.npz -- the TestRaftLogReadWrite scenario (TestRaftLogReadWrite.java:92-121):
    100 SimpleOperation entries, the expected file size (header + sum(varint(s)+s+4)) and the
    per-frame CRCs computed by the pinned CRC oracle.
"""
from __future__ import annotations

import hashlib
import json
import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as orc  # noqa: E402
from ratis_amd import segment  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
PJC = "/root/reference/ratis-common/src/main/java/org/apache/ratis/util/PureJavaCrc32C.java"

I64_MAX = (1 << 63) - 1
I64_MIN = -(1 << 63)

RFC3720 = [
    ("123456789", b"123456789", 0xE3069283),
    ("32 x 0x00", bytes(32), 0x8A9136AA),
    ("32 x 0xFF", b"\xff" * 32, 0x62A8AB43),
    ("0..31", bytes(range(32)), 0x46DD794E),
    ("31..0", bytes(range(31, -1, -1)), 0x113FDB5C),
]


def reference_table_sha256() -> str:
    src = open(PJC).read()
    body = src[src.index("private static final int[] T = new int[] {"):]
    body = body[:body.index("};")]
    vals = [int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]{8})", body)]
    assert len(vals) == 2048
    return hashlib.sha256(np.asarray(vals, dtype="<u4").tobytes()).hexdigest()


# (name, followers, in_new, in_old, include_self, transitional, include_self_old, self(flush), gap,
#  lastCommitted, term_start, expected getMajorityMin or None, expected commit after updateCommit)
CASES = [
    # 3 voters: sorted [7,10,12] -> majority s[1]=10; min(10, flush 12) = 10 >= termStart -> commit
    ("three_peers", [10, 7], [1, 1], [0, 0], 1, 0, 0, 12, -1, 5, 0, (7, 10, 12), 10),
    # 4 voters: sorted [3,5,8,9] -> s[(4-1)/2] = s[1] = 5 (3 of 4 voters have >= 5)
    ("even_quorum", [5, 9, 3], [1, 1, 1], [0, 0, 0], 1, 0, 0, 8, -1, 0, 0, (3, 5, 9), 5),
    # gap clamp: sorted [10,3000,3000], maj-min = 2990 > 1000 -> majority := min = 10
    ("gap_clamps", [10, 3000], [1, 1], [0, 0], 1, 0, 0, 3000, 1000, 0, 0, (10, 10, 3000), 10),
    # gap exactly at threshold: 1010-10 = 1000, not > 1000 -> no clamp
    ("gap_at_threshold", [10, 1010], [1, 1], [0, 0], 1, 0, 0, 2000, 1000, 0, 0, (10, 1010, 2000), 1010),
    # term check fails: newCommit 10 < termStart 11 (RaftLogBase.java:133-134)
    ("term_check_fails", [10, 7], [1, 1], [0, 0], 1, 0, 0, 12, -1, 5, 11, (7, 10, 12), 5),
    # term check passes exactly at termStart
    ("term_check_at_start", [10, 7], [1, 1], [0, 0], 1, 0, 0, 12, -1, 5, 10, (7, 10, 12), 10),
    # majority <= lastCommitted: no update (LeaderStateImpl.java:1017), min still reported
    ("no_progress", [10, 7], [1, 1], [0, 0], 1, 0, 0, 12, -1, 10, 0, (7, 10, 12), 10),
    # flushIndex clamp: sorted [15,20,20] -> maj 20; newCommit = min(20, flush 15) = 15
    ("flush_clamp", [20, 20], [1, 1], [0, 0], 1, 0, 0, 15, -1, 0, 0, (15, 20, 20), 15),
    # leader not in conf: sorted [4,6,8] -> maj 6; flushIndex still clamps (RaftLogBase.java:125)
    ("leader_not_voter", [4, 6, 8], [1, 1, 1], [0, 0, 0], 0, 0, 0, 100, -1, 0, 0, (4, 6, 8), 6),
    # follower without FollowerInfo / non-voter slot ignored: voters {f0, self} -> sorted [3,9] maj s[0]=3
    ("masked_follower", [3, 1000], [1, 0], [0, 0], 1, 0, 0, 9, -1, 0, 0, (3, 3, 9), 3),
    # fresh followers at -1: sorted [-1,-1,5] -> maj -1, not > lastCommitted -1
    ("fresh_followers", [-1, -1], [1, 1], [0, 0], 1, 0, 0, 5, -1, -1, 0, (-1, -1, 5), -1),
    # single-voter group (leader only): maj = flush
    ("leader_only", [], [], [], 1, 0, 0, 42, -1, 40, 0, (42, 42, 42), 42),
    # empty conf: no followers and leader not a voter -> Optional.empty() (LeaderStateImpl.java:964-966)
    ("empty_new_conf", [5, 6], [0, 0], [0, 0], 0, 0, 0, 9, -1, 0, 0, None, 0),
    # joint: new = {f0, f1, self}: [8,9,20] -> (8,9,20); old = {f1, f2, self}: [2,9,20] -> (2,9,20)
    # combine = element-wise min -> (2, 9, 20)
    ("joint_combine", [8, 9, 2], [1, 1, 0], [0, 1, 1], 1, 1, 1, 20, -1, 0, 0, (2, 9, 20), 9),
    # joint, old conf lags: new {f0,f1,self} [50,60,70] maj 60; old {f2,f3,self} [1,2,70] maj 2
    ("joint_old_lags", [50, 60, 1, 2], [1, 1, 0, 0], [0, 0, 1, 1], 1, 1, 1, 70, -1, 0, 0, (1, 2, 70), 2),
    # joint with an old conf that has no voter -> empty (LeaderStateImpl.java:976-978)
    ("joint_old_empty", [8, 9], [1, 1], [0, 0], 1, 1, 0, 20, -1, 0, 0, None, 0),
    # joint, leader only in old conf: new {f0,f1} [30,40] maj s[0]=30; old {f0, self} [30,35] maj 30
    ("joint_leader_leaving", [30, 40], [1, 1], [1, 0], 0, 1, 1, 35, -1, 0, 0, (30, 30, 35), 30),
    # Java long wrap in the gap test: maj - min = I64_MAX - (-1) wraps negative -> no clamp
    ("gap_wraps", [-1, I64_MAX], [1, 1], [0, 0], 1, 0, 0, I64_MAX, 5, 0, 0, (-1, I64_MAX, I64_MAX), I64_MAX),
]


# TestRaftLogIndex.testIndex: one RaftLogIndex("index", 900) driven through four sections; `i` is
# index.get() + 1 at the start of each section (TestRaftLogIndex.java:53, 61, 69, 77).  Each step:
# (op, argument, expected `updated`, expected index after, throws).  The updateIncreasingly section
# ends with the failure case (:56-57): getAndSet runs before the precondition throws, so the index
# is left at i - 1 = 900 and the updateToMax section starts from 900 (`updated` is never returned
# there: None).
RAFT_LOG_INDEX = [
    ("updateIncreasingly", 900, [("set", 901, True, 901, False), ("set", 901, False, 901, False),
                                 ("set", 900, None, 900, True)]),
    ("updateToMax", 900, [("set", 901, True, 901, False), ("set", 901, False, 901, False),
                          ("set", 900, False, 901, False)]),
    ("setUnconditionally", 901, [("set", 902, True, 902, False), ("set", 902, False, 902, False),
                                 ("set", 901, True, 901, False)]),
    ("updateUnconditionally", 901, [("add", 1, True, 902, False), ("add", 0, False, 902, False),
                                    ("add", -1, True, 901, False)]),
]

# TestPeerConfiguration: voters (self "0" first), then the assertions of :51-54 and :64-69.
PEER_CONFIGURATION = [
    {"name": "testOddNodesQuorum", "voters": ["0", "1", "2"], "self": "0",
     "has_majority": [{"others": ["1"], "expected": True}],
     "majority_reject_votes": [{"rejected": ["1"], "expected": False}]},
    {"name": "testEvenNodeQuorum", "voters": ["0", "1", "2", "3"], "self": "0",
     "has_majority": [{"others": ["1"], "expected": False}, {"others": ["1", "2"], "expected": True}],
     "majority_reject_votes": [{"rejected": ["1"], "expected": False}, {"rejected": ["1", "2"], "expected": True}]},
]


def raft_log_index_step(kind: str, old: int, op: str, arg: int):
    """RaftLogIndex.java:45-86 restated: returns (updated, new value, throws)."""
    if kind == "updateIncreasingly":      # getAndSet, then Preconditions.assertTrue(old <= new)
        return old != arg, arg, not old <= arg
    if kind == "updateToMax":             # getAndUpdate(max), updated = old < new
        return old < arg, max(old, arg), False
    if kind == "setUnconditionally":      # getAndSet, updated = old != new
        return old != arg, arg, False
    new = old + arg                       # updateUnconditionally(n -> n + arg)
    return old != new, new, False


def peer_has_majority(voters, others, self_id):
    """PeerConfiguration.hasMajority(others, selfId) (:152-169): num > size / 2."""
    num = (1 if self_id in voters else 0) + sum(1 for p in voters if p in others)
    return num > len(voters) // 2


def peer_majority_reject_votes(voters, rejected):
    """PeerConfiguration.majorityRejectVotes (:175-183): size - |rejected in conf| <= size / 2."""
    return len(voters) - sum(1 for p in rejected if p in voters) <= len(voters) // 2


def reference_sequences() -> dict:
    seqs = []
    for kind, init, steps in RAFT_LOG_INDEX:
        v = init
        out = []
        for op, arg, upd, after, throws in steps:
            got = raft_log_index_step(kind, v, op, arg)
            assert (None if throws else got[0], got[1], got[2]) == (upd, after, throws), (kind, op, arg, got)
            v = after
            out.append({"op": op, "arg": arg, "updated": upd, "after": after, "throws": throws})
        seqs.append({"method": kind, "initial": init, "steps": out})
    for c in PEER_CONFIGURATION:
        for h in c["has_majority"]:
            assert peer_has_majority(c["voters"], h["others"], c["self"]) == h["expected"], (c["name"], h)
        for r in c["majority_reject_votes"]:
            assert peer_majority_reject_votes(c["voters"], r["rejected"]) == r["expected"], (c["name"], r)
    return {"source": {"raft_log_index": "ratis-test/.../server/raftlog/TestRaftLogIndex.java:44-83",
                       "peer_configuration": "ratis-test/.../server/impl/TestPeerConfiguration.java:45-70"},
            "raft_log_index": seqs, "peer_configuration": PEER_CONFIGURATION}


def main():
    json.dump(reference_sequences(), open(os.path.join(HERE, "reference_sequences.json"), "w"), indent=1)

    # ---- CRC -------------------------------------------------------------------------------
    tab = orc.crc32c_tables()
    ours = hashlib.sha256(tab.astype("<u4").tobytes()).hexdigest()
    ref = reference_table_sha256()
    assert ours == ref, "generated slicing table differs from PureJavaCrc32C.java T[]"
    for name, data, want in RFC3720:
        assert orc.crc32c(data) == want == orc.crc32c_py(data), name
    json.dump({"table_sha256": ref, "table_source": "PureJavaCrc32C.java:167-688 (T8_0..T8_7, little-endian u32)",
               "rfc3720": [{"name": n, "hex": d.hex(), "crc": f"0x{c:08X}"} for n, d, c in RFC3720]},
              open(os.path.join(HERE, "crc_reference.json"), "w"), indent=1)

    # ---- commit ----------------------------------------------------------------------------
    out = []
    for (name, f, a, b, inc, tr, inco, self_v, gap, lc, ts, exp, exp_commit) in CASES:
        got_c = orc.get_majority_min(f, a, b, inc, tr, inco, self_v, gap)
        got_p = orc.py_get_majority_min(f, a, b, inc, tr, inco, self_v, gap)
        assert got_c == got_p == (tuple(exp) if exp else None), (name, got_c, got_p, exp)
        commit = lc
        if exp is not None:
            # literal two-term log [0, flush]: term 2 from termStart on, term 1 before
            flush = self_v
            n_terms = max(0, min(flush, 1 << 16) + 1)
            terms = [2 if i >= ts else 1 for i in range(n_terms)] if flush < (1 << 16) else []
            if terms:
                commit, _, _ = orc.update_commit(lc, exp[1], exp[0], flush, 2, 0, terms)
            else:  # huge indices: pointwise rule (same predicate)
                nc = min(exp[1], flush)
                if exp[1] > lc and lc < nc <= flush and nc >= ts:
                    commit = nc
        assert commit == exp_commit, (name, commit, exp_commit)
        out.append({"name": name, "followers": f, "in_new": a, "in_old": b, "include_self": inc,
                    "transitional": tr, "include_self_old": inco, "self_index": self_v, "gap": gap,
                    "last_committed": lc, "term_start": ts,
                    "expected": None if exp is None else {"min": exp[0], "majority": exp[1], "max": exp[2]},
                    "expected_commit": exp_commit})
    json.dump({"source": "hand-derived from LeaderStateImpl.java:904-1026 and RaftLogBase.java:121-142",
               "cases": out}, open(os.path.join(HERE, "commit_cases.json"), "w"), indent=1)

    # ---- TestRaftLogReadWrite scenario -------------------------------------------------------
    protos = segment.simple_operation_entries(100, term=0)
    img, offs, lens = segment.build_segment(protos)
    frames = [orc.frame_write(p) for p in protos]
    expect_size = len(segment.HEADER) + sum(segment.varint_size(len(p)) + len(p) + 4 for p in protos)
    img2 = np.frombuffer(segment.HEADER + b"".join(frames), dtype=np.uint8)
    assert img2.size == expect_size == img.size
    crcs, bad = orc.crc32c_frames(img2, offs, lens)
    assert bad == 0
    np.savez(os.path.join(HERE, "raftlog_rw.npz"), image=img2, frame_off=offs, frame_len=lens, crc=crcs,
             expected_size=np.int64(expect_size))
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
