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
    L.orc_has_lease.restype = c_int
    L.orc_has_lease.argtypes = [c_int, c_int64, c_int64, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int,
                                c_int64, POINTER(c_int64), POINTER(c_int)]
    L.orc_lease_soa.restype = None
    L.orc_lease_soa.argtypes = [c_uint64, c_uint32, c_int64, c_int64] + [c_void_p] * 7
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


def crc32c_frames_all(buf: np.ndarray, off: np.ndarray, frame_len: np.ndarray, threads: int = 16):
    """Every frame's PureJavaCrc32C over [off, off + len - 4) and whether it differs from the stored
    big-endian trailer (SegmentedRaftLogReader.decodeEntry, RDR:327-336), on `threads` host threads
    (ctypes releases the GIL; static slices).  Returns (crc uint32 [n], bad bool [n]).  The full
    config-5 parity check: every frame of the 8 GiB image, independent of how it was stamped."""
    import threading
    buf = np.ascontiguousarray(buf, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    ln = np.ascontiguousarray(frame_len, dtype=np.uint32)
    n = off.size
    crc = np.zeros(n, dtype=np.uint32)
    L = load()
    cuts = np.linspace(0, n, threads + 1).astype(np.int64)

    def run(a, b):
        if b > a:
            L.orc_crc32c_frames(_p(buf), _p(off[a:b]), _p(ln[a:b]), b - a, _p(crc[a:b]))
    th = [threading.Thread(target=run, args=(int(a), int(b))) for a, b in zip(cuts[:-1], cuts[1:])]
    for t in th:
        t.start()
    for t in th:
        t.join()
    end = (off + ln.astype(np.uint64)).astype(np.int64)
    stored = ((buf[end - 4].astype(np.uint32) << 24) | (buf[end - 3].astype(np.uint32) << 16)
              | (buf[end - 2].astype(np.uint32) << 8) | buf[end - 1].astype(np.uint32))
    return crc, crc != stored


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


# ---- leader lease ----------------------------------------------------------------------------
def has_lease(enabled: bool, now: int, timeout_ms: int, cur_ts, self_in_cur: bool, old_ts, self_in_old: bool,
              transitional: bool, lease_in: int):
    """orc_has_lease: LeaderStateImpl.hasLease for one group -> (has_lease, lease_out, extended)."""
    cur = np.ascontiguousarray(cur_ts if len(cur_ts) else [0], dtype=np.int64)
    old = np.ascontiguousarray(old_ts if len(old_ts) else [0], dtype=np.int64)
    lo, ext = c_int64(), c_int()
    r = load().orc_has_lease(int(enabled), now, timeout_ms, _p(cur), len(cur_ts), int(self_in_cur), _p(old),
                             len(old_ts), int(self_in_old), int(transitional), lease_in, ctypes.byref(lo),
                             ctypes.byref(ext))
    return bool(r), lo.value, bool(ext.value)


def py_has_lease(enabled, now, timeout_ms, cur_ts, self_in_cur, old_ts, self_in_old, transitional, lease_in):
    """Pure-Python restatement of LeaderStateImpl.hasLease (LSI:1229-1249) / LeaderLease (LL:60-103)
    with Java long semantics, written independently of the C one to cross-check it."""
    import functools

    def wrap(x):
        x &= (1 << 64) - 1
        return x - (1 << 64) if x >> 63 else x

    def cmp(a, b):                       # Timestamp.compareTo
        d = wrap(a - b)
        return (d > 0) - (d < 0)

    def elapsed_ms(t):                   # Timestamp.elapsedTimeMs, truncating division
        d = wrap(now - t)
        return abs(d) // 1000000 * (1 if d >= 0 else -1)

    def has_majority(active, include_self):   # PeerConfiguration.hasMajority
        if not active and not include_self:
            return True
        return (int(include_self) + sum(active)) > (len(active) + int(include_self)) // 2

    def max_ts(ts):                      # LeaderLease.getMaxTimestampWithMajorityAck
        if not ts:
            return now
        return sorted(ts, key=functools.cmp_to_key(cmp))[len(ts) // 2]

    if not enabled:
        return False, lease_in, False
    singleton = len(cur_ts) + int(self_in_cur) == 1 and \
        ((len(old_ts) + int(self_in_old)) if transitional else 0) <= 1
    if singleton or elapsed_ms(lease_in) < timeout_ms:
        return True, lease_in, False
    ok = has_majority([elapsed_ms(t) < timeout_ms for t in cur_ts], self_in_cur)
    if transitional:
        ok = ok and has_majority([elapsed_ms(t) < timeout_ms for t in old_ts], self_in_old)
    lease, ext = lease_in, False
    if ok:
        a = max_ts(list(cur_ts))
        b = max_ts(list(old_ts)) if transitional else now
        lease, ext = (b if cmp(a, b) > 0 else a), True
    return bool(singleton or elapsed_ms(lease) < timeout_ms), lease, ext


def lease_soa(follower_ts: np.ndarray, conf: np.ndarray, lease_in: np.ndarray, now: int, timeout_ms: int,
              enabled_bits: Optional[np.ndarray] = None):
    """Batched restatement with the argument layout of rh_lease_soa.  Returns a dict."""
    F, n = follower_ts.shape
    follower_ts = np.ascontiguousarray(follower_ts, dtype=np.int64)
    conf = np.ascontiguousarray(conf).astype(np.uint32)
    lease_in = np.ascontiguousarray(lease_in, dtype=np.int64)
    en = None if enabled_bits is None else np.ascontiguousarray(enabled_bits, dtype=np.uint64)
    lease_out = np.zeros(n, dtype=np.int64)
    nw = (n + 63) // 64
    hb = np.zeros(max(nw, 1), dtype=np.uint64)
    eb = np.zeros(max(nw, 1), dtype=np.uint64)
    load().orc_lease_soa(n, F, now, timeout_ms, _p(follower_ts), _p(conf), _p(lease_in), _p(en), _p(lease_out),
                         _p(hb), _p(eb))
    return {"lease": lease_out, "has_lease_bits": hb[:nw], "extended_bits": eb[:nw]}


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
