"""RaftGroupTable: the resident per-GPU table of leader divisions (``rh_groups`` in the C ABI).

This is the object the Java ``ratis-hip`` module holds.  Its methods mirror the
reference's producers and consumers of the commit index, batched over every group of the table:

  =============================================  ============================================
  reference (ratis tree)                         RaftGroupTable
  =============================================  ============================================
  FollowerInfo.updateMatchIndex                  :meth:`update_match_index` (monotone max)
    FollowerInfoImpl.java:93-95
  FollowerInfo.updateCommitIndex                 :meth:`update_follower_commit_index`
    FollowerInfoImpl.java:103-105
  SegmentedRaftLogWorker flush-index advance     :meth:`update_flush_index`
    SegmentedRaftLogWorker.java:419-431
  RaftConfigurationImpl change / leader start    :meth:`set_group`
    LeaderStateImpl.java:296-301, 624-633
  LeaderStateImpl.updateCommit()                 :meth:`update_commit`
    LeaderStateImpl.java:946-950, 1015-1026
  LeaderStateImpl.commitIndexChanged()           :meth:`commit_index_changed`
    LeaderStateImpl.java:612-622
  =============================================  ============================================

Host arrays are numpy; all compute is the HIP kernel behind ``rh_commit_batch`` /
``rh_watch_levels``.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _lib
from ._lib import RhDelta, check


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class RaftGroupTable:
    def __init__(self, ctx, capacity: int, n_followers: int, gap_threshold: int = -1):
        self._lib = _lib.load()
        self.ctx = ctx
        self.capacity = int(capacity)
        self.n_followers = int(n_followers)
        self.gap_threshold = int(gap_threshold)
        h = ctypes.c_void_p()
        check(self._lib.rh_groups_create(ctx.handle, self.capacity, self.n_followers, self.gap_threshold,
                                         ctypes.byref(h)))
        self._h = h

    # -- lifecycle --------------------------------------------------------------------------
    def close(self) -> None:
        if self._h is not None:
            check(self._lib.rh_groups_destroy(self._h))
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        if self._h is None:
            raise _lib.RatisHipError(_lib.RH_E_STATE, "RaftGroupTable closed")
        return self._h

    # -- conf / bulk load -------------------------------------------------------------------
    def set_group(self, slot: int, conf: int, flush_index: int, commit_index: int, term_start: int) -> None:
        check(self._lib.rh_group_set(self.handle, slot, conf & 0xFFFFFFFF, flush_index, commit_index, term_start))

    def load(self, first: int, n: int, match: Optional[np.ndarray] = None, fcommit: Optional[np.ndarray] = None,
             flush: Optional[np.ndarray] = None, commit: Optional[np.ndarray] = None,
             term_start: Optional[np.ndarray] = None, conf: Optional[np.ndarray] = None) -> None:
        def i64(a, shape):
            if a is None:
                return None
            a = np.ascontiguousarray(a, dtype=np.int64)
            if a.shape != shape:
                raise ValueError(f"expected shape {shape}, got {a.shape}")
            return a

        F = self.n_followers
        match = i64(match, (F, n))
        fcommit = i64(fcommit, (F, n))
        flush, commit, term_start = i64(flush, (n,)), i64(commit, (n,)), i64(term_start, (n,))
        if conf is not None:
            conf = np.ascontiguousarray(conf).astype(np.uint32)
            if conf.shape != (n,):
                raise ValueError("conf shape")
        check(self._lib.rh_groups_load(self.handle, first, n, _p(match), _p(fcommit), _p(flush), _p(commit),
                                       _p(term_start), _p(conf)))

    # -- delta producers --------------------------------------------------------------------
    def push_deltas(self, slots: np.ndarray, columns: np.ndarray, values: np.ndarray) -> None:
        slots = np.asarray(slots, dtype=np.uint64)
        n = slots.size
        arr = np.zeros(n, dtype=[("slot", "<u8"), ("column", "<u4"), ("reserved", "<u4"), ("value", "<i8")])
        arr["slot"] = slots
        arr["column"] = np.broadcast_to(np.asarray(columns, dtype=np.uint32), (n,))
        arr["value"] = np.broadcast_to(np.asarray(values, dtype=np.int64), (n,))
        ptr = arr.ctypes.data_as(ctypes.POINTER(RhDelta))
        check(self._lib.rh_push_deltas(self.handle, ptr, n))

    DELTA_DTYPE = np.dtype([("slot", "<u8"), ("column", "<u4"), ("reserved", "<u4"), ("value", "<i8")])

    def acquire_deltas(self) -> np.ndarray:
        """Zero-copy producer path: the next pinned staging slot as a structured numpy array
        (fields slot/column/reserved/value) to fill in place; hand it over with
        :meth:`submit_deltas`.  The view is valid only until that call."""
        ptr = ctypes.c_void_p()
        cap = ctypes.c_size_t()
        check(self._lib.rh_deltas_acquire(self.handle, ctypes.byref(ptr), ctypes.byref(cap)))
        raw = (ctypes.c_uint8 * (cap.value * self.DELTA_DTYPE.itemsize)).from_address(ptr.value)
        return np.frombuffer(raw, dtype=self.DELTA_DTYPE)

    def submit_deltas(self, n: int) -> None:
        """Enqueues H2D + device apply of the first ``n`` deltas of the acquired slot (async)."""
        check(self._lib.rh_deltas_submit(self.handle, int(n)))

    def update_match_index(self, slots, follower_slot: int, values) -> None:
        self.push_deltas(slots, _lib.rh_col_match(follower_slot), values)

    def update_follower_commit_index(self, slots, follower_slot: int, values) -> None:
        self.push_deltas(slots, _lib.rh_col_fcommit(follower_slot), values)

    def update_flush_index(self, slots, values) -> None:
        self.push_deltas(slots, _lib.RH_COL_FLUSH, values)

    # -- consumers --------------------------------------------------------------------------
    def update_commit(self, want_min: bool = False) -> Tuple[np.ndarray, np.ndarray, Optional[np.ndarray]]:
        """Batched ``LeaderStateImpl.updateCommit()``: returns (slots, new commit index) of the
        groups whose commit index advanced (sorted by slot), and optionally the watch-ALL
        level (``min``) of every slot (INT64_MIN where getMajorityMin is empty)."""
        cap = self.capacity
        slots = np.empty(cap, dtype=np.uint64)
        commits = np.empty(cap, dtype=np.int64)
        mins = np.empty(cap, dtype=np.int64) if want_min else None
        n = ctypes.c_size_t()
        check(self._lib.rh_commit_batch(self.handle, _p(slots), _p(commits), cap, ctypes.byref(n), _p(mins)))
        k = n.value
        order = np.argsort(slots[:k], kind="stable")
        return slots[:k][order], commits[:k][order], mins

    def commit_index_changed(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
        """Batched ``commitIndexChanged()`` levels: (min, majority, max, valid[bool])."""
        cap = self.capacity
        mn, mj, mx = (np.empty(cap, dtype=np.int64) for _ in range(3))
        bits = np.empty((cap + 63) // 64, dtype=np.uint64)
        check(self._lib.rh_watch_levels(self.handle, _p(mn), _p(mj), _p(mx), _p(bits)))
        valid = np.unpackbits(bits.view(np.uint8), bitorder="little")[:cap].astype(bool)
        return mn, mj, mx, valid

    def read_commit(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.capacity - first if n is None else n
        out = np.empty(n, dtype=np.int64)
        check(self._lib.rh_groups_read_commit(self.handle, first, n, _p(out)))
        return out
