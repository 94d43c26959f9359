"""Parity oracle -- TEST INFRASTRUCTURE ONLY.

Python access to the C restatement (oracle/ratis_oracle.c -> oracle/_build/libratis_oracle.so)
plus a second, independent pure-Python restatement of the commit arithmetic used to
cross-check the C one on small cases.  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product (ratis_amd/) never does.

Reference citations (ratis tree):
  LeaderStateImpl.java:904-984, 1015-1026, 1076-1095   commit arithmetic
  RaftLogBase.java:121-142                             updateCommitIndex
  PureJavaCrc32C.java:43-152                           CRC32C
  SegmentedRaftLogOutputStream.java:86-110             frame writer
  SegmentedRaftLogReader.java:179-341                  frame reader
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from ctypes import POINTER, c_int, c_int64, c_size_t, c_uint32, c_uint64, c_void_p
from typing import List, Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "libratis_oracle.so")

ORC_OK, ORC_END, ORC_PARTIAL = 0, 1, 2
ORC_E_OVERSIZE, ORC_E_CHECKSUM, ORC_E_PADDING, ORC_E_VARINT, ORC_E_HEADER = -1, -2, -3, -4, -5

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    L = ctypes.CDLL(LIB)
    L.orc_crc32c.restype = c_uint32
    L.orc_crc32c.argtypes = [c_void_p, c_size_t]
    L.orc_crc32c_update_array.restype = c_uint32
    L.orc_crc32c_update_array.argtypes = [c_uint32, c_void_p, c_size_t, c_size_t]
    L.orc_crc32c_update_bytebuffer.restype = c_uint32
    L.orc_crc32c_update_bytebuffer.argtypes = [c_uint32, c_void_p, c_size_t, c_size_t]
    L.orc_crc32c_tables.argtypes = [c_void_p]
    L.orc_crc32c_frames.restype = c_uint64
    L.orc_crc32c_frames.argtypes = [c_void_p, c_void_p, c_void_p, c_uint64, c_void_p]
    L.orc_get_majority_min.restype = c_int
    L.orc_get_majority_min.argtypes = [c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_int64,
                                       c_int64, c_void_p]
    L.orc_update_commit_index.restype = c_int
    L.orc_update_commit_index.argtypes = [POINTER(c_int64), c_int64, c_int64, c_int64, c_int64, c_void_p, c_int64]
    L.orc_update_commit.restype = c_int
    L.orc_update_commit.argtypes = [POINTER(c_int64), c_int64, c_int64, c_int64, c_int64, c_int64, c_void_p,
                                    c_int64, POINTER(c_int64)]
    L.orc_commit_soa.restype = None
    L.orc_commit_soa.argtypes = [c_uint64, c_uint32, c_int, c_int64] + [c_void_p] * 12
    L.orc_varint32_size.restype = c_int
    L.orc_varint32_size.argtypes = [c_uint32]
    L.orc_frame_write.restype = c_uint32
    L.orc_frame_write.argtypes = [c_void_p, c_void_p, c_uint32]
    L.orc_decode_entry.restype = c_int
    L.orc_decode_entry.argtypes = [c_void_p, c_uint64, c_uint64, c_uint32, POINTER(c_uint32), POINTER(c_uint32),
                                   POINTER(c_uint32), POINTER(c_uint64)]
    L.orc_verify_header.restype = c_int
    L.orc_verify_header.argtypes = [c_void_p, c_uint64]
    L.orc_segment_scan.restype = c_uint64
    L.orc_segment_scan.argtypes = [c_void_p, c_uint64, c_uint32, c_uint64, c_void_p, c_void_p, c_void_p,
                                   POINTER(c_int), POINTER(c_uint64)]
    _lib = L
    return L


def _p(a):
    return None if a is None else a.ctypes.data_as(c_void_p)


# ---- CRC32C ----------------------------------------------------------------------------------
def crc32c(data: bytes) -> int:
    """getValue() of a fresh PureJavaCrc32C after update(data, 0, len)."""
    b = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    return load().orc_crc32c(_p(b), len(data))


def crc32c_update(state: int, data: bytes, bytebuffer: bool = False) -> int:
    """PureJavaCrc32C.update on the internal (bit-flipped) state; returns the new state."""
    b = np.frombuffer(bytes(data), dtype=np.uint8) if len(data) else np.zeros(1, np.uint8)
    f = load().orc_crc32c_update_bytebuffer if bytebuffer else load().orc_crc32c_update_array
    return f(state & 0xFFFFFFFF, _p(b), 0, len(data))


def crc32c_tables() -> np.ndarray:
    t = np.zeros(2048, dtype=np.uint32)
    load().orc_crc32c_tables(_p(t))
    return t


def crc32c_frames(buf: np.ndarray, off: np.ndarray, frame_len: np.ndarray) -> Tuple[np.ndarray, int]:
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(frame_len, dtype=np.uint32)
    out = np.zeros(off.size, dtype=np.uint32)
    bad = load().orc_crc32c_frames(_p(buf), _p(off), _p(ln), off.size, _p(out))
    return out, int(bad)


def crc32c_py(data: bytes, state: int = 0xFFFFFFFF) -> int:
    """Bit-at-a-time CRC-32C (reflected 0x82F63B78), a third, table-free restatement."""
    c = state
    for b in data:
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0x82F63B78 if c & 1 else 0)
    return (~c) & 0xFFFFFFFF


# ---- commit ----------------------------------------------------------------------------------
def get_majority_min(vals: Sequence[int], in_new: Sequence[int], in_old: Sequence[int], include_self: bool,
                     transitional: bool, include_self_old: bool, self_val: int, gap: int) -> Optional[Tuple[int, int, int]]:
    nf = len(vals)
    v = np.asarray(vals, dtype=np.int64)
    a = np.asarray(in_new, dtype=np.uint8)
    b = np.asarray(in_old, dtype=np.uint8)
    out = np.zeros(3, dtype=np.int64)
    ok = load().orc_get_majority_min(_p(v) if nf else None, nf, _p(a) if nf else None, _p(b) if nf else None,
                                     int(include_self), int(transitional), int(include_self_old), self_val, gap,
                                     _p(out))
    return (int(out[0]), int(out[1]), int(out[2])) if ok == 1 else None


def _wrap64(x: int) -> int:
    x = int(x) & ((1 << 64) - 1)
    return x - (1 << 64) if x >> 63 else x


def py_get_majority_min(vals, in_new, in_old, include_self, transitional, include_self_old, self_val, gap):
    """Pure-Python restatement of LeaderStateImpl.getMajorityMin (LeaderStateImpl.java:956-984)."""
    vals = [int(v) for v in vals]
    self_val = int(self_val)

    def sorted_of(member, inc):
        xs = [vals[i] for i in range(len(vals)) if member[i]]
        if inc:
            xs.append(self_val)
        return sorted(xs)

    def value_of(s):
        maj = s[(len(s) - 1) // 2]
        mn = s[0]
        if gap != -1 and _wrap64(maj - mn) > gap:
            maj = mn
        return mn, maj, s[-1]

    if not any(in_new) and not include_self:
        return None
    r = value_of(sorted_of(in_new, include_self))
    if not transitional:
        return r
    if not any(in_old) and not include_self_old:
        return None
    o = value_of(sorted_of(in_old, include_self_old))
    return tuple(min(x, y) for x, y in zip(r, o))


def update_commit(commit_index: int, majority: int, mn: int, flush: int, current_term: int, log_start: int,
                  terms: Sequence[int]) -> Tuple[int, bool, int]:
    """LSI:1015-1026 + RLB:121-142 with a literal term array; returns (commit, advanced, watch_all)."""
    t = np.asarray(terms, dtype=np.int64) if len(terms) else np.zeros(1, np.int64)
    c = c_int64(commit_index)
    w = c_int64(0)
    adv = load().orc_update_commit(ctypes.byref(c), majority, mn, flush, current_term, log_start, _p(t), len(terms),
                                   ctypes.byref(w))
    return c.value, bool(adv), w.value


def commit_soa(follower: np.ndarray, self_index: np.ndarray, conf: np.ndarray, mode: int = 0, gap: int = -1,
               commit_in: Optional[np.ndarray] = None, term_start: Optional[np.ndarray] = None,
               log_start: Optional[np.ndarray] = None):
    """Batched restatement with the argument layout of rh_commit_soa.  Returns a dict."""
    F, n = follower.shape
    follower = np.ascontiguousarray(follower, dtype=np.int64)
    self_index = np.ascontiguousarray(self_index, dtype=np.int64)
    conf = np.ascontiguousarray(conf).astype(np.uint32)
    commit_in = np.ascontiguousarray(commit_in if commit_in is not None else np.zeros(n), dtype=np.int64)
    term_start = np.ascontiguousarray(term_start if term_start is not None else np.zeros(n), dtype=np.int64)
    ls = None if log_start is None else np.ascontiguousarray(log_start, dtype=np.int64)
    out = {k: np.zeros(n, dtype=np.int64) for k in ("commit", "min", "maj", "max")}
    nw = (n + 63) // 64
    vb = np.zeros(nw, dtype=np.uint64)
    ab = np.zeros(nw, dtype=np.uint64)
    load().orc_commit_soa(n, F, mode, gap, _p(follower), _p(self_index), _p(commit_in), _p(term_start), _p(ls),
                          _p(conf), _p(out["commit"]), _p(out["min"]), _p(out["maj"]), _p(out["max"]), _p(vb),
                          _p(ab))
    out["valid_bits"] = vb
    out["advanced_bits"] = ab
    return out


# ---- frames ----------------------------------------------------------------------------------
def frame_write(proto: bytes) -> bytes:
    dst = np.zeros(len(proto) + 9, dtype=np.uint8)
    src = np.frombuffer(proto, dtype=np.uint8) if proto else np.zeros(1, np.uint8)
    n = load().orc_frame_write(_p(dst), _p(src), len(proto))
    return dst[:n].tobytes()


def decode_entry(seg: np.ndarray, pos: int, max_op: int = 4 << 20):
    seg = np.ascontiguousarray(seg, dtype=np.uint8)
    el, cc, cs, nx = c_uint32(), c_uint32(), c_uint32(), c_uint64()
    st = load().orc_decode_entry(_p(seg), seg.size, pos, max_op, ctypes.byref(el), ctypes.byref(cc), ctypes.byref(cs),
                                 ctypes.byref(nx))
    return st, el.value, cc.value, cs.value, nx.value


def segment_scan(seg: np.ndarray, max_op: int = 4 << 20, cap: int = 1 << 20):
    seg = np.ascontiguousarray(seg, dtype=np.uint8)
    offs = np.zeros(cap, dtype=np.uint64)
    lens = np.zeros(cap, dtype=np.uint32)
    crcs = np.zeros(cap, dtype=np.uint32)
    st = c_int()
    stop = c_uint64()
    n = load().orc_segment_scan(_p(seg), seg.size, max_op, cap, _p(offs), _p(lens), _p(crcs), ctypes.byref(st),
                                ctypes.byref(stop))
    k = min(n, cap)
    return offs[:k].astype(np.int64), lens[:k].astype(np.int32), crcs[:k], st.value, stop.value
