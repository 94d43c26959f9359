"""RaftGroupTable / RaftNode: the resident per-GPU table of leader divisions (``rh_groups``) and the
multi-GPU server built from them (``rh_node``), include/ratis_hip.h.

This is the object the Java ``ratis-hip`` module holds.  Its methods mirror the
reference's producers and consumers of the commit index, batched over every division of a
server (paths relative to the ratis tree, ratis-server/.../server/impl/ unless noted):

  ==============================================  ===========================================
  reference                                       RaftGroupTable
  ==============================================  ===========================================
  new LeaderStateImpl: addSenders, StartupLogEntry :meth:`start`
    LeaderStateImpl.java:296-301, 421-430, 681-692
  applyOldNewConf / replicateNewConf / restart    :meth:`reconf`
    LeaderStateImpl.java:624-633, 704-724, 1064-1074
  step down / group removal                       :meth:`stop`
  FollowerInfo.updateMatchIndex                   :meth:`update_match_index` (RH_OP_MAX)
    FollowerInfoImpl.java:93-95
  FollowerInfo.setSnapshotIndex                   :meth:`set_snapshot_index` (RH_OP_SET)
    FollowerInfoImpl.java:147-151
  FollowerInfo.updateCommitIndex                  :meth:`update_follower_commit_index`
    FollowerInfoImpl.java:103-105
  SegmentedRaftLogWorker flush-index advance      :meth:`update_flush_index`
    raftlog/segmented/SegmentedRaftLogWorker.java:419-431
  LeaderStateImpl.updateCommit() (dirty groups)   :meth:`update_commit`, :meth:`commit_async`
    LeaderStateImpl.java:946-950, 1015-1026
  LeaderStateImpl.commitIndexChanged()            :meth:`commit_index_changed`
    LeaderStateImpl.java:606-622
  ==============================================  ===========================================

Host arrays are numpy; all compute is the HIP kernels behind the calls.  Errors raise
``_lib.IllegalArgumentError`` for RH_E_INVAL / RH_E_RANGE (Java: IllegalArgumentException) and
``_lib.RatisHipError`` otherwise.
"""
from __future__ import annotations

import ctypes
import threading
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import RhCommitOut, check

DELTA_DTYPE = np.dtype([("slot", "<u4"), ("column", "u1"), ("op", "u1"), ("reserved", "<u2"), ("value", "<i8")])
INDEX_EVENT_DTYPE = np.dtype([("slot", "<u4"), ("reserved", "<u4"), ("value", "<i8")])
WATCH_EVENT_DTYPE = np.dtype([("slot", "<u4"), ("valid", "<u4"), ("min", "<i8"), ("majority", "<i8"), ("max", "<i8")])


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _view(ptr: int, n: int, dtype: np.dtype) -> np.ndarray:
    if n == 0 or not ptr:
        return np.zeros(0, dtype=dtype)
    raw = (ctypes.c_uint8 * (n * dtype.itemsize)).from_address(ptr)
    return np.frombuffer(raw, dtype=dtype)


def make_deltas(slots, columns, values, ops=_lib.RH_OP_MAX) -> np.ndarray:
    """Structured array of ``rh_delta`` (16 bytes each)."""
    slots = np.asarray(slots, dtype=np.uint32).reshape(-1)
    n = slots.size
    d = np.zeros(n, dtype=DELTA_DTYPE)
    d["slot"] = slots
    d["column"] = np.broadcast_to(np.asarray(columns, dtype=np.uint8), (n,))
    d["op"] = np.broadcast_to(np.asarray(ops, dtype=np.uint8), (n,))
    d["value"] = np.broadcast_to(np.asarray(values, dtype=np.int64), (n,))
    return d


def _src_array(src: Optional[Sequence[int]]):
    if src is None:
        return None
    a = np.full(_lib.RH_MAX_FOLLOWERS, -1, dtype=np.int8)
    s = np.asarray(src, dtype=np.int64)
    a[: s.size] = s
    return a


def _addr(a: np.ndarray):
    """The array's address for a ``void*`` argument: a ctypes reference to its buffer (a pump tick's
    push is a few microseconds; ``ndarray.ctypes.data_as`` alone costs 2-4 of them), or, for a
    read-only or empty array, ``ndarray.ctypes.data``."""
    try:
        return ctypes.byref(ctypes.c_char.from_buffer(a))
    except (TypeError, ValueError):
        return a.ctypes.data


class CommitResult:
    """Events of one batched updateCommit: copies of the library's pinned result buffers."""

    def __init__(self, out: RhCommitOut):
        adv = _view(out.advanced or 0, out.n_advanced, INDEX_EVENT_DTYPE)
        wall = _view(out.watch_all or 0, out.n_watch_all, INDEX_EVENT_DTYPE)
        o = np.argsort(adv["slot"], kind="stable")
        self.advanced_slots = adv["slot"][o].astype(np.int64)
        self.advanced_commit = adv["value"][o].copy()
        o = np.argsort(wall["slot"], kind="stable")
        self.watch_all_slots = wall["slot"][o].astype(np.int64)
        self.watch_all_min = wall["value"][o].copy()


class RaftGroupTable:
    def __init__(self, ctx, capacity: int, gap_threshold: int = -1):
        self._lib = _lib.load()
        self.ctx = ctx
        self.capacity = int(capacity)
        self.gap_threshold = int(gap_threshold)
        h = ctypes.c_void_p()
        check(self._lib.rh_groups_create(ctx.handle, self.capacity, self.gap_threshold, ctypes.byref(h)))
        self._h = h

    @classmethod
    def _wrap(cls, handle, capacity: int, gap_threshold: int):
        t = cls.__new__(cls)
        t._lib = _lib.load()
        t.ctx = None
        t.capacity = capacity
        t.gap_threshold = gap_threshold
        t._h = ctypes.c_void_p(handle)
        t._owned = False
        return t

    # -- lifecycle --------------------------------------------------------------------------
    def close(self) -> None:
        h, self._h = self._h, None
        if h is not None and getattr(self, "_owned", True):
            check(self._lib.rh_groups_destroy(h))   # raises if the table's last work faulted

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        if self._h is None:
            raise _lib.RatisHipError(_lib.RH_E_STATE, "RaftGroupTable closed")
        return self._h

    def set_event_sink(self, sink: int) -> None:
        """``rh_groups_set_event_sink``: RH_EVENTS_HOST_MAPPED (kernel writes events across PCIe,
        the default) or RH_EVENTS_DEVICE (events staged in HBM, copied out by the wait)."""
        check(self._lib.rh_groups_set_event_sink(self.handle, int(sink)))

    # -- control ----------------------------------------------------------------------------
    def start(self, slot: int, conf: int, flush_index: int, commit_index: int, term_start: int) -> None:
        check(self._lib.rh_group_start(self.handle, slot, conf & 0xFFFFFFFF, flush_index, commit_index, term_start))

    def reconf(self, slot: int, conf: int, src: Optional[Sequence[int]] = None) -> None:
        a = _src_array(src)
        check(self._lib.rh_group_reconf(self.handle, slot, conf & 0xFFFFFFFF, _p(a)))

    def stop(self, slot: int) -> None:
        check(self._lib.rh_group_stop(self.handle, slot))

    def tier_width(self, slot: int) -> int:
        w = ctypes.c_uint32()
        check(self._lib.rh_group_tier(self.handle, slot, ctypes.byref(w)))
        return w.value

    def load(self, first: int, conf: np.ndarray, flush: np.ndarray, commit: np.ndarray, term_start: np.ndarray,
             match: Optional[np.ndarray] = None, fcommit: Optional[np.ndarray] = None) -> None:
        """Bulk start of slots [first, first + n) with explicit follower state ([F, n] arrays)."""
        conf = np.ascontiguousarray(conf).astype(np.uint32)
        n = conf.size
        f = 0
        arrs = []
        for a in (match, fcommit):
            if a is not None:
                a = np.ascontiguousarray(a, dtype=np.int64)
                if a.ndim != 2 or a.shape[1] != n:
                    raise ValueError("match / fcommit must be [F, n]")
                f = max(f, a.shape[0])
            arrs.append(a)
        match, fcommit = arrs
        if match is not None and fcommit is not None and match.shape != fcommit.shape:
            raise ValueError("match and fcommit shapes differ")
        cols = [np.ascontiguousarray(x, dtype=np.int64) for x in (flush, commit, term_start)]
        if any(c.shape != (n,) for c in cols):
            raise ValueError("flush / commit / term_start must be [n]")
        check(self._lib.rh_groups_load(self.handle, first, n, f, _p(match), _p(fcommit), _p(cols[0]), _p(cols[1]),
                                       _p(cols[2]), _p(conf)))

    # -- delta producers --------------------------------------------------------------------
    def push(self, deltas: np.ndarray) -> None:
        deltas = np.ascontiguousarray(deltas, dtype=DELTA_DTYPE)
        check(self._lib.rh_push_deltas(self.handle, _addr(deltas), deltas.size))

    def push_deltas(self, slots, columns, values, ops=_lib.RH_OP_MAX) -> None:
        self.push(make_deltas(slots, columns, values, ops))

    def update_match_index(self, slots, follower_slot: int, values) -> None:
        self.push_deltas(slots, _lib.rh_col_match(follower_slot), values)

    def set_snapshot_index(self, slots, follower_slot: int, values) -> None:
        """FollowerInfo.setSnapshotIndex: matchIndex set unconditionally (may go down)."""
        self.push_deltas(slots, _lib.rh_col_match(follower_slot), values, _lib.RH_OP_SET)

    def update_follower_commit_index(self, slots, follower_slot: int, values) -> None:
        self.push_deltas(slots, _lib.rh_col_fcommit(follower_slot), values)

    def update_flush_index(self, slots, values) -> None:
        self.push_deltas(slots, _lib.RH_COL_FLUSH, values)

    def acquire_deltas(self) -> np.ndarray:
        """Zero-copy producer path: the next pinned staging slot as a structured numpy array to
        fill in place; hand it over with :meth:`submit_deltas`.  Valid only until that call."""
        ptr = ctypes.c_void_p()
        cap = ctypes.c_size_t()
        check(self._lib.rh_deltas_acquire(self.handle, ctypes.byref(ptr), ctypes.byref(cap)))
        return _view(ptr.value, cap.value, DELTA_DTYPE)

    def submit_deltas(self, n: int) -> None:
        """Enqueues H2D + device apply of the first ``n`` deltas of the acquired slot (async)."""
        check(self._lib.rh_deltas_submit(self.handle, int(n)))

    # -- consumers --------------------------------------------------------------------------
    def commit_async(self, watch_all: bool = True) -> int:
        tk = ctypes.c_uint64()
        check(self._lib.rh_commit_batch_async(self.handle, _lib.RH_COMMIT_WATCH_ALL if watch_all else 0,
                                              ctypes.byref(tk)))
        return tk.value

    def commit_wait(self, ticket: int) -> CommitResult:
        out = RhCommitOut()
        check(self._lib.rh_commit_batch_wait(self.handle, ticket, ctypes.byref(out)))
        return CommitResult(out)

    def commit_wait_counts(self, ticket: int) -> Tuple[int, int]:
        """Like :meth:`commit_wait` but returns only (n_advanced, n_watch_all): the events stay in
        the library's pinned buffers (the bench's pipelined loop)."""
        out = RhCommitOut()
        check(self._lib.rh_commit_batch_wait(self.handle, ticket, ctypes.byref(out)))
        return int(out.n_advanced), int(out.n_watch_all)

    def update_commit(self, watch_all: bool = True) -> CommitResult:
        """Batched ``LeaderStateImpl.updateCommit()`` over the dirty slots: the slots whose commit
        index advanced (sorted, with the new value) and, with ``watch_all``, the slots whose
        watch-ALL level changed."""
        out = RhCommitOut()
        check(self._lib.rh_commit_batch(self.handle, _lib.RH_COMMIT_WATCH_ALL if watch_all else 0,
                                        ctypes.byref(out)))
        return CommitResult(out)

    def commit_index_changed(self) -> np.ndarray:
        """Batched ``commitIndexChanged()``: the changed levels (WATCH_EVENT_DTYPE, sorted by slot)."""
        ptr = ctypes.c_void_p()
        n = ctypes.c_uint64()
        check(self._lib.rh_watch_levels(self.handle, ctypes.byref(ptr), ctypes.byref(n)))
        ev = _view(ptr.value or 0, n.value, WATCH_EVENT_DTYPE).copy()
        return ev[np.argsort(ev["slot"], kind="stable")]

    def set_timing(self, enable: bool = True) -> None:
        """``rh_groups_timing``: HIP events around every evaluation (its kernels, events included)."""
        check(self._lib.rh_groups_timing(self.handle, 1 if enable else 0))

    def last_timing(self) -> float:
        """Device ms of the last timed evaluation (``rh_groups_last_timing``)."""
        a = ctypes.c_float()
        check(self._lib.rh_groups_last_timing(self.handle, ctypes.byref(a), None))
        return float(a.value)

    def last_timing_split(self) -> dict:
        """``rh_groups_last_timing_split``: the last timed _async split in submit (staged deltas' H2D +
        apply), eval (the evaluation kernels), events (until the records are in the pinned lists) and
        gather (the REGION gather kernel alone, 0 if none), device ms; ``list``: whether it ran over the
        dirty-row lists; ``fused``: both kinds in one launch (:meth:`tick_async`)."""
        a, b, c, d, m = ctypes.c_float(), ctypes.c_float(), ctypes.c_float(), ctypes.c_float(), ctypes.c_int()
        check(self._lib.rh_groups_last_timing_split(self.handle, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c),
                                                    ctypes.byref(d), ctypes.byref(m)))
        return {"submit_ms": float(a.value), "eval_ms": float(b.value), "events_ms": float(c.value),
                "gather_ms": float(d.value), "list": bool(m.value), "fused": m.value == 2}

    def last_was_list(self) -> bool:
        """Whether the last (timed) evaluation ran over the dirty-row lists (list mode)."""
        a, m = ctypes.c_float(), ctypes.c_int()
        check(self._lib.rh_groups_last_timing(self.handle, ctypes.byref(a), ctypes.byref(m)))
        return bool(m.value)

    def watch_async(self) -> None:
        """``rh_watch_levels_async``: commitIndexChanged() of the dirty slots, in flight."""
        check(self._lib.rh_watch_levels_async(self.handle))

    def tick_async(self, watch_all: bool = True) -> int:
        """``rh_tick_async``: :meth:`commit_async` then :meth:`watch_async` in one call (one kernel
        launch when both kinds run over their dirty-row lists); collect with :meth:`commit_wait` (the
        returned ticket) and :meth:`watch_wait`."""
        tk = ctypes.c_uint64()
        check(self._lib.rh_tick_async(self.handle, _lib.RH_COMMIT_WATCH_ALL if watch_all else 0, ctypes.byref(tk)))
        return tk.value

    def watch_wait(self) -> np.ndarray:
        """``rh_watch_levels_wait``: the outstanding evaluation's changed levels, sorted by slot."""
        ptr = ctypes.c_void_p()
        n = ctypes.c_uint64()
        check(self._lib.rh_watch_levels_wait(self.handle, ctypes.byref(ptr), ctypes.byref(n)))
        ev = _view(ptr.value or 0, n.value, WATCH_EVENT_DTYPE).copy()
        return ev[np.argsort(ev["slot"], kind="stable")]

    def watch_wait_count(self) -> int:
        """Like :meth:`watch_wait` but returns only the number of changed levels: the events stay in
        the library's pinned list (the bench's pipelined loop)."""
        ptr = ctypes.c_void_p()
        n = ctypes.c_uint64()
        check(self._lib.rh_watch_levels_wait(self.handle, ctypes.byref(ptr), ctypes.byref(n)))
        return int(n.value)

    # -- leader lease (LeaderStateImpl.hasLease, LeaderLease) ---------------------------------
    def lease_start(self, slot: int, now_nanos: int, enabled: bool = True) -> None:
        """A new LeaderLease for ``slot`` (lease = now, enabled) with every follower stamped now."""
        check(self._lib.rh_group_lease_start(self.handle, int(slot), int(now_nanos), 1 if enabled else 0))

    def update_last_responded(self, slots, follower_slot: int, send_times) -> None:
        """FollowerInfo.updateLastRespondedAppendEntriesSendTime (a Timestamp set)."""
        self.push_deltas(slots, _lib.RH_COL_TS(follower_slot), send_times, ops=_lib.RH_OP_SET)

    def set_lease_enabled(self, slots, enabled: bool) -> None:
        """LeaderLease.getAndSetEnabled (step-down, leader not in the new conf)."""
        n = np.size(slots)
        self.push_deltas(slots, _lib.RH_COL_LEASE_ON, np.full(n, 1 if enabled else 0, np.int64), ops=_lib.RH_OP_SET)

    def lease_batch(self, now_nanos: int, timeout_ms: int) -> np.ndarray:
        """hasLease() (less isRunning()/isReady()) of every slot at now: bool [capacity]; extended
        leases are stored in the table."""
        ptr = ctypes.c_void_p()
        words = ctypes.c_uint64()
        check(self._lib.rh_lease_batch(self.handle, int(now_nanos), int(timeout_ms), ctypes.byref(ptr),
                                       ctypes.byref(words)))
        w = _view(ptr.value, words.value, np.dtype(np.uint64)).copy()
        return np.unpackbits(w.view(np.uint8), bitorder="little")[: self.capacity].astype(bool)

    def lease_async(self, now_nanos: int, timeout_ms: int) -> None:
        """``rh_lease_batch_async``: the hasLease pass in flight."""
        check(self._lib.rh_lease_batch_async(self.handle, int(now_nanos), int(timeout_ms)))

    def lease_wait(self) -> np.ndarray:
        """``rh_lease_batch_wait``: the outstanding pass's bitmap, bool [capacity]."""
        ptr = ctypes.c_void_p()
        words = ctypes.c_uint64()
        check(self._lib.rh_lease_batch_wait(self.handle, ctypes.byref(ptr), ctypes.byref(words)))
        w = _view(ptr.value, words.value, np.dtype(np.uint64)).copy()
        return np.unpackbits(w.view(np.uint8), bitorder="little")[: self.capacity].astype(bool)

    def read(self, column: int, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        n = self.capacity - first if n is None else n
        out = np.empty(n, dtype=np.int64)
        check(self._lib.rh_groups_read(self.handle, first, n, column, _p(out)))
        return out

    def read_commit(self, first: int = 0, n: Optional[int] = None) -> np.ndarray:
        return self.read(_lib.RH_COL_COMMITTED, first, n)


def shard_of(msb: int, lsb: int, n_shards: int) -> int:
    """``rh_shard_of``: floorMod(RaftGroupId.hashCode(), n) computed by the library."""
    return check(_lib.load().rh_shard_of(msb & (2**64 - 1), lsb & (2**64 - 1), n_shards))


class RaftNode:
    """``rh_node``: one RaftServer's leader divisions over every GPU of ``device_mask`` -- or, with
    ``devices``, one shard per listed device (repeats allowed: several shards on one GPU)."""

    def __init__(self, device_mask: int, capacity_per_shard: int, gap_threshold: int = -1,
                 devices: Optional[Sequence[int]] = None):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        if devices is not None:
            arr = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            check(self._lib.rh_node_create_devices(arr, len(devices), capacity_per_shard, gap_threshold,
                                                   ctypes.byref(h)))
        else:
            check(self._lib.rh_node_create(device_mask, capacity_per_shard, gap_threshold, ctypes.byref(h)))
        self._h = h
        self.capacity_per_shard = int(capacity_per_shard)
        self.n_shards = check(self._lib.rh_node_shards(h))
        self.tables = [RaftGroupTable._wrap(self._lib.rh_node_groups(h, s), capacity_per_shard, gap_threshold)
                       for s in range(self.n_shards)]

    def close(self) -> None:
        h, self._h = self._h, None
        if h is not None:
            check(self._lib.rh_node_destroy(h))

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def place(self, msb: int, lsb: int, index_in_shard: int) -> int:
        """Node slot of a RaftGroupId: its shard's base + the module's slot within that shard."""
        return shard_of(msb, lsb, self.n_shards) * self.capacity_per_shard + index_in_shard

    def start(self, node_slot: int, conf: int, flush_index: int, commit_index: int, term_start: int) -> None:
        check(self._lib.rh_node_group_start(self._h, node_slot, conf & 0xFFFFFFFF, flush_index, commit_index,
                                            term_start))

    def reconf(self, node_slot: int, conf: int, src: Optional[Sequence[int]] = None) -> None:
        check(self._lib.rh_node_group_reconf(self._h, node_slot, conf & 0xFFFFFFFF, _p(_src_array(src))))

    def stop(self, node_slot: int) -> None:
        check(self._lib.rh_node_group_stop(self._h, node_slot))

    def push(self, deltas: np.ndarray) -> None:
        deltas = np.ascontiguousarray(deltas, dtype=DELTA_DTYPE)
        check(self._lib.rh_node_push_deltas(self._h, _addr(deltas), deltas.size))

    def update_commit(self, cap: int) -> Tuple[np.ndarray, np.ndarray]:
        """All shards' updateCommit events: (advanced, watch_all) structured arrays, node slots."""
        adv = np.zeros(cap, dtype=INDEX_EVENT_DTYPE)
        wall = np.zeros(cap, dtype=INDEX_EVENT_DTYPE)
        na, nw = ctypes.c_uint64(), ctypes.c_uint64()
        check(self._lib.rh_node_commit_batch(self._h, _lib.RH_COMMIT_WATCH_ALL, _p(adv), cap, ctypes.byref(na),
                                             _p(wall), cap, ctypes.byref(nw)))
        a = adv[: min(na.value, cap)]
        w = wall[: min(nw.value, cap)]
        return a[np.argsort(a["slot"], kind="stable")], w[np.argsort(w["slot"], kind="stable")]

    def watch_levels(self, cap: int) -> np.ndarray:
        """All shards' commitIndexChanged() level changes (node slots), sorted by slot."""
        out = np.zeros(max(cap, 1), dtype=WATCH_EVENT_DTYPE)
        n = ctypes.c_uint64()
        check(self._lib.rh_node_watch_levels(self._h, _p(out), cap, ctypes.byref(n)))
        ev = out[: min(n.value, cap)]
        return ev[np.argsort(ev["slot"], kind="stable")]

    def lease_start(self, node_slot: int, now_nanos: int, enabled: bool = True) -> None:
        check(self._lib.rh_node_group_lease_start(self._h, node_slot, int(now_nanos), 1 if enabled else 0))

    def lease_batch(self, now_nanos: int, timeout_ms: int) -> np.ndarray:
        """hasLease() of every node slot (bool [n_shards * capacity_per_shard])."""
        total = self.n_shards * self.capacity_per_shard
        bits = np.zeros((total + 63) // 64, dtype=np.uint64)
        check(self._lib.rh_node_lease_batch(self._h, int(now_nanos), int(timeout_ms), _p(bits), bits.size))
        return np.unpackbits(bits.view(np.uint8), bitorder="little")[:total].astype(bool)


class _DeltaBuffer:
    """One producer thread's deltas (HipLeaderBookkeeper.DeltaBuffer): appended under its own lock,
    pushed whole when full or when the pump / a control call flushes every buffer."""

    CAP = 4096

    def __init__(self, node: "RaftNode"):
        self.node = node
        self.lock = threading.Lock()
        self.parts: List[np.ndarray] = []
        self.n = 0

    def put(self, deltas: np.ndarray) -> None:
        with self.lock:
            self.parts.append(deltas)
            self.n += deltas.size
            if self.n >= self.CAP:
                self._flush_locked()

    def flush(self) -> None:
        with self.lock:
            self._flush_locked()

    def _flush_locked(self) -> None:
        if self.parts:
            self.node.push(np.concatenate(self.parts))
            self.parts, self.n = [], 0


class LeaderPump:
    """Python twin of the Java module's pump (java/ratis-hip/.../HipLeaderBookkeeper.tick): one
    tick = push every producer thread's buffered deltas; put every shard's updateCommit, commitIndexChanged() and (with
    a lease timeout) hasLease pass in flight -- all shards before any wait; then per shard hand the
    advanced commits and watch-ALL levels to the divisions, then commitIndexChanged()'s levels
    (LeaderStateImpl.java:606-622), then the lease bitmap.  ``callbacks[node_slot]`` gets
    ``on_commit(value)``, ``on_watch_all(min)`` and ``on_watch_levels(min, majority, max)`` (the
    last only for a present getMajorityMin, as commitIndexChanged's ifPresent)."""

    def __init__(self, node: RaftNode, lease_timeout_ms: int = -1):
        self.node = node
        self.callbacks = {}
        self._buffers: List[_DeltaBuffer] = []   # one per producer thread (thread-local)
        self._local = threading.local()
        self._reg = threading.Lock()
        self.lease_timeout_ms = lease_timeout_ms
        self.lease_bits = None
        self.fallbacks = {}   # reason -> divisions that left the table (HipLeaderBookkeeper.getFallbackCount)

    def register(self, node_slot: int, callback) -> None:
        self.callbacks[int(node_slot)] = callback

    def emit(self, deltas: np.ndarray) -> None:
        b = getattr(self._local, "buf", None)
        if b is None:
            b = self._local.buf = _DeltaBuffer(self.node)
            with self._reg:
                self._buffers.append(b)
        b.put(np.ascontiguousarray(deltas, dtype=DELTA_DTYPE))

    def drain(self) -> None:
        """Pushes every producer's buffered deltas now (HipLeaderBookkeeper.flushAllDeltas: each tick,
        and before a control call)."""
        with self._reg:
            bufs = list(self._buffers)
        for b in bufs:
            b.flush()

    def division(self, node_slot: int, callback) -> "PumpDivision":
        d = PumpDivision(self, int(node_slot), callback)
        self.register(node_slot, callback)
        return d

    def tick(self, now_nanos: int = 0) -> dict:
        self.drain()
        cap = self.node.capacity_per_shard
        lease = self.lease_timeout_ms >= 0
        tickets = []
        for t in self.node.tables:   # every shard's passes in flight before any wait (stream order:
            tickets.append(t.tick_async(watch_all=True))   # commit, then its commitIndexChanged)
            if lease:
                t.lease_async(now_nanos, self.lease_timeout_ms)
        n = {"commit": 0, "watch_all": 0, "watch_levels": 0}
        bits = []
        for s, (t, tk) in enumerate(zip(self.node.tables, tickets)):
            r = t.commit_wait(tk)
            for slot, v in zip(r.advanced_slots, r.advanced_commit):
                cb = self.callbacks.get(s * cap + int(slot))
                if cb is not None:
                    cb.on_commit(int(v))
                    n["commit"] += 1
            for slot, v in zip(r.watch_all_slots, r.watch_all_min):
                cb = self.callbacks.get(s * cap + int(slot))
                if cb is not None:
                    cb.on_watch_all(int(v))
                    n["watch_all"] += 1
            for e in t.watch_wait():
                if not e["valid"]:
                    continue
                cb = self.callbacks.get(s * cap + int(e["slot"]))
                if cb is not None:
                    cb.on_watch_levels(int(e["min"]), int(e["majority"]), int(e["max"]))
                    n["watch_levels"] += 1
            if lease:
                bits.append(t.lease_wait())
        self.lease_bits = np.concatenate(bits) if lease else None
        return n


class PumpDivision:
    """Python twin of HipLeaderBookkeeper.Division: the division's follower slots (addFollower,
    first free slot of 14), its membership word, its control calls and producers, and FALLBACK --
    a 15th follower (or a control call the library rejects) makes the division leave the table:
    its slot is stopped, later deltas are dropped, no event reaches it, the pump counts it and
    ``callback.on_fallback()`` runs (the reference's own per-division path from then on)."""

    MAX_FOLLOWERS = 14

    def __init__(self, pump: LeaderPump, node_slot: int, callback):
        self.pump, self.node_slot, self.callback = pump, node_slot, callback
        self.follower_slot = {}
        self.started = False
        self.fallback = False
        self.width = 0

    def fall_back(self, reason: str) -> None:
        if self.fallback:
            return
        self.fallback = True
        if self.started:
            self.started = False
            self.pump.drain()
            self.pump.node.stop(self.node_slot)
        self.pump.callbacks.pop(self.node_slot, None)
        self.pump.fallbacks[reason] = self.pump.fallbacks.get(reason, 0) + 1
        if hasattr(self.callback, "on_fallback"):
            self.callback.on_fallback()

    def _emit(self, follower: int, column: int, op: int, value: int) -> None:
        if not self.started or self.fallback or follower >= self.width:
            return
        self.pump.emit(make_deltas([self.node_slot], [column], [value], op))

    def add_follower(self, peer) -> int:
        if self.fallback:
            return -1
        if peer in self.follower_slot:
            return self.follower_slot[peer]
        used = set(self.follower_slot.values())
        for k in range(self.MAX_FOLLOWERS):
            if k not in used:
                self.follower_slot[peer] = k
                self._reset_slot(k)
                return k
        self.fall_back("FOLLOWER_SLOTS")
        return -1

    def _reset_slot(self, k: int) -> None:
        """A new FollowerInfo (-1, -1) on slot k, ordered after every delta of the slot's previous
        occupant in any producer's buffer (HipLeaderBookkeeper.resetFollowerSlot): every buffer is
        pushed first, then the SETs go straight to the node, not through this thread's buffer."""
        if not self.started or self.fallback or k >= self.width:
            return
        self.pump.drain()
        self.pump.node.push(make_deltas([self.node_slot] * 2, [_lib.rh_col_match(k), _lib.rh_col_fcommit(k)],
                                        [-1, -1], _lib.RH_OP_SET))

    def remove_follower(self, peer) -> None:
        """The peer's buffered deltas pushed now: none can follow the next occupant's reset."""
        self.follower_slot.pop(peer, None)
        if self.started and not self.fallback:
            self.pump.drain()

    def conf_word(self, conf, old=None, self_in_conf=True, self_in_old=True) -> int:
        n = sum(1 << self.follower_slot[p] for p in conf if p in self.follower_slot)
        o = sum(1 << self.follower_slot[p] for p in (old or ()) if p in self.follower_slot)
        return _lib.conf_pack(n, self_in_conf, old is not None, o, old is not None and self_in_old, True)

    @staticmethod
    def _width(conf: int) -> int:
        m = (conf & 0x3FFF) | ((conf >> 16) & 0x3FFF)
        w = m.bit_length()
        return 2 if w <= 2 else 2 * ((w + 1) // 2)

    def start(self, conf: int, flush: int, commit: int, term_start: int) -> None:
        if self.fallback:
            return
        self.pump.drain()
        try:
            self.pump.node.start(self.node_slot, conf, flush, commit, term_start)
        except _lib.RatisHipError:
            self.fall_back("REJECTED")
            return
        self.width = self._width(conf)
        self.started = True

    def reconf(self, conf: int) -> None:
        if not self.started or self.fallback:
            return
        self.pump.drain()
        try:
            self.pump.node.reconf(self.node_slot, conf)
        except _lib.RatisHipError:
            self.fall_back("REJECTED")
            return
        self.width = self._width(conf)

    def match_index(self, k: int, v: int) -> None:
        if k >= 0:
            self._emit(k, _lib.rh_col_match(k), _lib.RH_OP_MAX, v)

    def follower_commit_index(self, k: int, v: int) -> None:
        if k >= 0:
            self._emit(k, _lib.rh_col_fcommit(k), _lib.RH_OP_MAX, v)

    def flush_index(self, v: int) -> None:
        self._emit(-1, _lib.RH_COL_FLUSH, _lib.RH_OP_MAX, v)
