"""Device-side host API: contexts, commit tiers and frame batches over torch-owned HBM.

PyTorch is used only as plumbing here -- device memory (``torch.empty(..., device='cuda')``)
and streams (``torch.cuda.current_stream()``).  Every computation is a libratis_hip kernel
reached through the C ABI in ``include/ratis_hip.h``.

Reference mapping (paths relative to the ratis tree):
  * :func:`commit_launch` with ``mode=COMMIT`` = ``LeaderStateImpl.updateCommit()``
    (LeaderStateImpl.java:946-950, 956-984, 1015-1026) + ``RaftLogBase.updateCommitIndex``
    (RaftLogBase.java:121-142), for every group of every tier.
  * ``mode=WATCH`` = ``LeaderStateImpl.commitIndexChanged()`` (LeaderStateImpl.java:612-622).
  * :func:`crc32c_frames` = ``PureJavaCrc32C`` (PureJavaCrc32C.java:43-152) over
    ``SegmentedRaftLogOutputStream.write`` frames (:86-110), verified as in
    ``SegmentedRaftLogReader.decodeEntry`` (:327-336) or stamped as in the writer.
  * :func:`lease_launch` = ``LeaderStateImpl.hasLease()`` (LeaderStateImpl.java:1229-1249) with
    ``LeaderLease.extend`` (LeaderLease.java:68-103) for every group of every tier.
  * :func:`segments_scan` = the reader's framing walk (``verifyHeader`` :179-205, ``decodeEntry``
    :291-323, ``verifyTerminator`` :251-280) over many segment images at once, and
    :func:`read_segments` = framing + CRC verify, i.e. ``LogSegment.readSegmentFile``
    (LogSegment.java:166-196) minus the proto parse.
"""
from __future__ import annotations

import ctypes
import weakref
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import torch

from . import _lib
from ._lib import RH_MODE_COMMIT, RH_MODE_WATCH, RhCommitSoa, RhFrames, RhLeaseSoa, RhSegments, RhSegmentsCrc, check


def _ptr(t: Optional[torch.Tensor]) -> Optional[int]:
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("expected a CUDA (HIP) tensor")
    if not t.is_contiguous():
        raise ValueError("expected a contiguous tensor")
    return t.data_ptr()


def _stream_ptr(stream: Optional[torch.cuda.Stream]) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


_LIVE = weakref.WeakSet()


def live_contexts() -> List["Context"]:
    """The contexts not closed yet (tests/conftest.py drains each after every GPU test)."""
    return [c for c in list(_LIVE) if c._h is not None]


class Context:
    """One ``rh_ctx`` per (process, GPU)."""

    def __init__(self, device: int = 0):
        lib = _lib.load()
        if not torch.cuda.is_available():
            raise RuntimeError("ratis_amd.Context needs a GPU (MI355X/gfx950); there is no CPU fallback")
        self.device = device
        torch.cuda.set_device(device)
        h = ctypes.c_void_p()
        check(lib.rh_init(device, ctypes.byref(h)))
        self._h = h
        _LIVE.add(self)

    @property
    def handle(self) -> ctypes.c_void_p:
        if self._h is None:
            raise _lib.RatisHipError(_lib.RH_E_STATE, "context closed")
        return self._h

    def synchronize(self) -> None:
        """``rh_synchronize``: the context stream drained, an outstanding zero-copy stamp settled;
        raises on a fault of that work."""
        check(_lib.load().rh_synchronize(self.handle))

    def close(self) -> None:
        if self._h is not None:
            h, self._h = self._h, None
            check(_lib.load().rh_shutdown(h))   # raises if the context's last work faulted

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


# ------------------------------------------------------------------------------------------
# Quorum commit
# ------------------------------------------------------------------------------------------
@dataclass
class CommitTier:
    """One struct-of-arrays tier on the device (all tensors CUDA, contiguous).

    ``follower_index`` is ``[F, n]`` int64 (row k = follower slot k), ``conf`` is int32 holding
    the uint32 membership words of ``ratis_hip.h``.
    """

    follower_index: torch.Tensor
    self_index: torch.Tensor
    conf: torch.Tensor
    commit_in: Optional[torch.Tensor] = None
    term_start: Optional[torch.Tensor] = None
    commit_out: Optional[torch.Tensor] = None
    min_out: Optional[torch.Tensor] = None
    maj_out: Optional[torch.Tensor] = None
    max_out: Optional[torch.Tensor] = None
    valid_bits: Optional[torch.Tensor] = None
    advanced_bits: Optional[torch.Tensor] = None
    gap_threshold: int = -1
    adv_rows: Optional[torch.Tensor] = None
    adv_commit: Optional[torch.Tensor] = None
    adv_count: Optional[torch.Tensor] = None
    adv_row_base: int = 0

    @property
    def n(self) -> int:
        return int(self.self_index.numel())

    @property
    def n_followers(self) -> int:
        return int(self.follower_index.shape[0])

    def alloc_outputs(self, mode: int = RH_MODE_COMMIT, levels: bool = False, bits: bool = True) -> "CommitTier":
        dev = self.self_index.device
        n = self.n
        nw = (n + 63) // 64
        if mode == RH_MODE_COMMIT and self.commit_out is None:
            self.commit_out = torch.empty(n, dtype=torch.int64, device=dev)
        if self.min_out is None:
            self.min_out = torch.empty(n, dtype=torch.int64, device=dev)
        if levels or mode == RH_MODE_WATCH:
            if self.maj_out is None:
                self.maj_out = torch.empty(n, dtype=torch.int64, device=dev)
            if self.max_out is None:
                self.max_out = torch.empty(n, dtype=torch.int64, device=dev)
        if bits:
            if self.valid_bits is None:
                self.valid_bits = torch.zeros(nw, dtype=torch.int64, device=dev)
            if mode == RH_MODE_COMMIT and self.advanced_bits is None:
                self.advanced_bits = torch.zeros(nw, dtype=torch.int64, device=dev)
        return self

    def to_struct(self, mode: int) -> RhCommitSoa:
        fi = self.follower_index
        if fi.dim() != 2 or fi.dtype != torch.int64:
            raise ValueError("follower_index must be an int64 [F, n] tensor")
        n = self.n
        for name in ("self_index", "commit_in", "term_start", "commit_out", "min_out", "maj_out", "max_out"):
            t = getattr(self, name)
            if t is not None and (t.dtype != torch.int64 or t.numel() != n):
                raise ValueError(f"{name} must be int64 with {n} elements")
        if self.conf.dtype != torch.int32 or self.conf.numel() != n:
            raise ValueError("conf must be int32 (uint32 bit patterns) with n elements")
        s = RhCommitSoa()
        s.n = n
        s.n_followers = fi.shape[0]
        s.mode = mode
        s.gap_threshold = self.gap_threshold if mode == RH_MODE_COMMIT else -1
        if not fi.is_cuda or (fi.stride(1) != 1 and n > 1) or fi.stride(0) < n:
            raise ValueError("follower_index must be a CUDA [F, n] view with unit row stride")
        s.follower_index = fi.data_ptr()
        s.col_stride = fi.stride(0)
        s.self_index = _ptr(self.self_index)
        s.commit_in = _ptr(self.commit_in)
        s.term_start = _ptr(self.term_start)
        s.conf = _ptr(self.conf)
        s.commit_out = _ptr(self.commit_out)
        s.min_out = _ptr(self.min_out)
        s.maj_out = _ptr(self.maj_out)
        s.max_out = _ptr(self.max_out)
        s.valid_bits = _ptr(self.valid_bits)
        s.advanced_bits = _ptr(self.advanced_bits) if mode == RH_MODE_COMMIT else None
        if self.adv_rows is not None:
            s.adv_rows = _ptr(self.adv_rows)
            s.adv_commit = _ptr(self.adv_commit)
            s.adv_count = _ptr(self.adv_count)
            s.adv_cap = self.adv_rows.numel()
            s.adv_row_base = self.adv_row_base
        return s


@dataclass
class TiledCommitTier:
    """A commit tier in the TILED layout of ``rh_commit_soa.tile_stride``: one int64 HBM buffer of
    ceil(n / 128) tiles.  A tile holds, for its 128 groups, the F follower columns, self_index,
    commit_in, term_start, commit_out, min_out (and maj_out, max_out with ``levels``), 128 int64
    each, then the 128 uint32 membership words -- so a wave's loads are one contiguous run per
    tile.  Rows past n in the last tile are padding (never evaluated).  Bit columns stay plain."""

    n: int
    n_followers: int
    buf: torch.Tensor               # int64 [n_tiles, tile_elems]
    levels: bool = False
    gap_threshold: int = -1
    min_out: bool = True             # request the watch-ALL level column
    valid_bits: Optional[torch.Tensor] = None
    advanced_bits: Optional[torch.Tensor] = None

    @staticmethod
    def columns(F: int, levels: bool) -> List[str]:
        return [f"f{k}" for k in range(F)] + ["self", "commit_in", "term_start", "commit_out", "min_out"] + \
            (["maj_out", "max_out"] if levels else [])

    @classmethod
    def tile_elems(cls, F: int, levels: bool) -> int:
        return len(cls.columns(F, levels)) * 128 + 64  # + 128 uint32 conf words

    @classmethod
    def from_arrays(cls, follower, self_index, conf, commit_in, term_start, device="cuda", gap_threshold: int = -1,
                    levels: bool = False, bits: bool = True) -> "TiledCommitTier":
        import numpy as np
        F, n = follower.shape
        nt = (n + 127) // 128
        cols = cls.columns(F, levels)
        te = cls.tile_elems(F, levels)
        host = np.zeros((nt, te), dtype=np.int64)

        def put(name, a):
            c = cols.index(name)
            pad = np.zeros(nt * 128, dtype=np.int64)
            pad[:n] = a
            host[:, c * 128:(c + 1) * 128] = pad.reshape(nt, 128)
        for k in range(F):
            put(f"f{k}", follower[k])
        put("self", self_index)
        put("commit_in", commit_in)
        put("term_start", term_start)
        cw = np.zeros(nt * 128, dtype=np.uint32)
        cw[:n] = conf
        host[:, len(cols) * 128:] = cw.reshape(nt, 128).view(np.int64)
        t = cls(n=n, n_followers=F, buf=torch.from_numpy(host).to(device), levels=levels,
                gap_threshold=gap_threshold)
        if bits:
            nw = (n + 63) // 64
            t.valid_bits = torch.zeros(nw, dtype=torch.int64, device=device)
            t.advanced_bits = torch.zeros(nw, dtype=torch.int64, device=device)
        return t

    def column(self, name: str) -> torch.Tensor:
        """Column ``name`` over the n groups (a gathered copy)."""
        c = self.columns(self.n_followers, self.levels).index(name)
        return self.buf[:, c * 128:(c + 1) * 128].reshape(-1)[:self.n]

    def to_struct(self, mode: int) -> RhCommitSoa:
        cols = self.columns(self.n_followers, self.levels)
        base = self.buf.data_ptr()

        def at(name):
            return base + cols.index(name) * 128 * 8
        s = RhCommitSoa()
        s.n = self.n
        s.n_followers = self.n_followers
        s.mode = mode
        s.gap_threshold = self.gap_threshold if mode == RH_MODE_COMMIT else -1
        s.follower_index = at("f0")
        s.col_stride = 128
        s.self_index = at("self")
        s.commit_in = at("commit_in")
        s.term_start = at("term_start")
        s.conf = base + len(cols) * 128 * 8
        s.commit_out = at("commit_out") if mode == RH_MODE_COMMIT else None
        s.min_out = at("min_out") if self.min_out else None
        if self.levels:
            s.maj_out = at("maj_out")
            s.max_out = at("max_out")
        s.valid_bits = _ptr(self.valid_bits)
        s.advanced_bits = _ptr(self.advanced_bits) if mode == RH_MODE_COMMIT else None
        s.tile_stride = self.buf.shape[1] * 8
        return s


def commit_launch(ctx: Context, tiers: Sequence, mode: int = RH_MODE_COMMIT,
                  stream: Optional[torch.cuda.Stream] = None) -> None:
    """Enqueues one fused commit kernel over up to RH_MAX_TIERS tiers (asynchronous)."""
    if not 1 <= len(tiers) <= _lib.RH_MAX_TIERS:
        raise ValueError("1..4 tiers per launch")
    arr = (RhCommitSoa * len(tiers))(*[t.to_struct(mode) for t in tiers])
    check(_lib.load().rh_commit_soa_launch(ctx.handle, arr, len(tiers), _stream_ptr(stream)))


class PreparedLaunch:
    """A launch whose rh_*_soa argument arrays are built once (the tier buffers do not move between
    launches, as a long-lived host would hold them): calling it is one C-ABI call.  Rebuilding the
    ctypes structs per launch costs ~10-20 us of Python -- as long as a 1M-group lease or commit
    kernel, enough to leave the GPU waiting for the host."""

    def __init__(self, fn_name: str, *arrays_and_counts):
        self._fn = getattr(_lib.load(), fn_name)
        self._args = arrays_and_counts      # keeps the ctypes arrays alive

    def __call__(self, ctx: "Context", stream: Optional[torch.cuda.Stream] = None) -> None:
        check(self._fn(ctx.handle, *self._args, _stream_ptr(stream)))


def prepare_commit(tiers: Sequence, mode: int = RH_MODE_COMMIT) -> PreparedLaunch:
    """commit_launch with the argument array built once."""
    if not 1 <= len(tiers) <= _lib.RH_MAX_TIERS:
        raise ValueError("1..4 tiers per launch")
    return PreparedLaunch("rh_commit_soa_launch", (RhCommitSoa * len(tiers))(*[t.to_struct(mode) for t in tiers]),
                          len(tiers))


def unpack_bits(words: torch.Tensor, n: int) -> torch.Tensor:
    """Bit g of word g//64 -> bool tensor [n] (on the words' device)."""
    w = words.view(torch.int64)
    shifts = torch.arange(64, device=w.device, dtype=torch.int64)
    bits = (w.unsqueeze(1) >> shifts) & 1
    return bits.reshape(-1)[:n].bool()


# ------------------------------------------------------------------------------------------
# CRC32C over frames
# ------------------------------------------------------------------------------------------
@dataclass
class FrameBatch:
    """A segment image in HBM plus its frame table."""

    buf: torch.Tensor          # uint8 [buf_len]
    frame_off: torch.Tensor    # int64 [n]: offset of each frame's first varint byte
    frame_len: torch.Tensor    # int32 [n]: varint + proto + 4
    crc_out: Optional[torch.Tensor] = None   # int32 [n] (uint32 bit patterns)
    bad_bits: Optional[torch.Tensor] = None  # int64 [ceil(n/64)]
    n_bad: Optional[torch.Tensor] = None     # int64 [1]

    @property
    def n(self) -> int:
        return int(self.frame_off.numel())

    def alloc_outputs(self) -> "FrameBatch":
        dev = self.buf.device
        if self.crc_out is None:
            self.crc_out = torch.empty(self.n, dtype=torch.int32, device=dev)
        if self.bad_bits is None:
            self.bad_bits = torch.zeros((self.n + 63) // 64, dtype=torch.int64, device=dev)
        if self.n_bad is None:
            self.n_bad = torch.zeros(1, dtype=torch.int64, device=dev)
        return self

    def to_struct(self, init_state: int) -> RhFrames:
        if self.buf.dtype != torch.uint8:
            raise ValueError("buf must be uint8")
        if self.frame_off.dtype != torch.int64 or self.frame_len.dtype != torch.int32:
            raise ValueError("frame_off must be int64 and frame_len int32")
        if self.frame_len.numel() != self.n:
            raise ValueError("frame_off and frame_len lengths differ")
        f = RhFrames()
        f.buf = _ptr(self.buf)
        f.buf_len = self.buf.numel()
        f.frame_off = _ptr(self.frame_off)
        f.frame_len = _ptr(self.frame_len)
        f.n = self.n
        f.init_state = init_state & 0xFFFFFFFF
        f.crc_out = _ptr(self.crc_out)
        f.bad_bits = _ptr(self.bad_bits)
        f.n_bad = _ptr(self.n_bad)
        return f


def crc32c_frames(ctx: Context, batch: FrameBatch, flags: int = _lib.RH_CRC_VERIFY,
                  init_state: int = 0xFFFFFFFF, stream: Optional[torch.cuda.Stream] = None) -> None:
    """Enqueues the frame CRC kernel (asynchronous).  ``flags``: 0, RH_CRC_VERIFY or RH_CRC_STAMP."""
    f = batch.to_struct(init_state)
    check(_lib.load().rh_crc32c_frames_launch(ctx.handle, ctypes.byref(f), flags, _stream_ptr(stream)))


def crc32c_bytes(ctx: Context, data: torch.Tensor, init_state: int = 0xFFFFFFFF) -> int:
    """``PureJavaCrc32C`` state after ``update(data)`` from ``init_state``, as getValue() (uint32).

    One span, computed by the frame kernel with no trailer (flags = 0)."""
    if data.dtype != torch.uint8 or not data.is_cuda:
        raise ValueError("data must be a CUDA uint8 tensor")
    n = data.numel()
    buf = data if n else torch.zeros(1, dtype=torch.uint8, device=data.device)
    fb = FrameBatch(buf=buf,
                    frame_off=torch.zeros(1, dtype=torch.int64, device=data.device),
                    frame_len=torch.full((1,), n, dtype=torch.int32, device=data.device))
    fb.alloc_outputs()
    crc32c_frames(ctx, fb, flags=0, init_state=init_state)
    torch.cuda.synchronize()
    return int(fb.crc_out.item()) & 0xFFFFFFFF


def crc32c_update(ctx: Context, state: int, data: bytes) -> int:
    """``PureJavaCrc32C.update(byte[], 0, len)`` on the internal state through ``rh_crc32c`` (host span
    staged to the device).  Returns the new state; ``getValue() = ~state & 0xFFFFFFFF``."""
    lib = _lib.load()
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    out = ctypes.c_uint32()
    check(lib.rh_crc32c(ctx.handle, state & 0xFFFFFFFF, buf, len(data), ctypes.byref(out)))
    return out.value


def crc32c_update_host(state: int, data: bytes) -> int:
    """``rh_crc32c_update``: the same on the host (pure, no context or device; SURVEY 8(b)'s
    ``rh_crc32c``).  Returns the new state."""
    buf = ctypes.create_string_buffer(bytes(data), max(1, len(data)))
    return int(_lib.load().rh_crc32c_update(state & 0xFFFFFFFF, buf, len(data)))


# ---- segment framing ---------------------------------------------------------------------------
RH_SEG_E_CHECKSUM = -2   # read_segments only: the first frame whose CRC does not verify


@dataclass
class SegmentBatch:
    """Many segment images in one HBM buffer, plus the framing outputs."""

    buf: torch.Tensor          # uint8 [buf_len]
    seg_off: torch.Tensor      # int64 [n_seg]
    seg_len: torch.Tensor      # int64 [n_seg]
    max_op: int = 4 * 1024 * 1024
    frames_per_seg_cap: int = 4096
    frame_cap: Optional[int] = None
    scratch_off: Optional[torch.Tensor] = None
    scratch_len: Optional[torch.Tensor] = None
    frame_off: Optional[torch.Tensor] = None   # int64 [frame_cap]
    frame_len: Optional[torch.Tensor] = None   # int32 [frame_cap]
    seg_first: Optional[torch.Tensor] = None   # int64 [n_seg]
    seg_nframes: Optional[torch.Tensor] = None  # int32 [n_seg]
    seg_status: Optional[torch.Tensor] = None  # int32 [n_seg]
    seg_stop: Optional[torch.Tensor] = None    # int64 [n_seg]
    total_frames: Optional[torch.Tensor] = None  # int64 [1]

    @property
    def n_seg(self) -> int:
        return int(self.seg_off.numel())

    def alloc_outputs(self) -> "SegmentBatch":
        dev, n, cap = self.buf.device, self.n_seg, self.frames_per_seg_cap
        if self.frame_cap is None:
            self.frame_cap = max(1, n * cap)
        e = lambda k, dt: torch.empty(k, dtype=dt, device=dev)  # noqa: E731
        if self.scratch_off is None:
            self.scratch_off = e(max(1, n * cap), torch.int64)
            self.scratch_len = e(max(1, n * cap), torch.int32)
        if self.frame_off is None:
            self.frame_off = e(self.frame_cap, torch.int64)
            self.frame_len = e(self.frame_cap, torch.int32)
        if self.seg_first is None:
            self.seg_first = e(max(1, n), torch.int64)
            self.seg_nframes = e(max(1, n), torch.int32)
            self.seg_status = e(max(1, n), torch.int32)
            self.seg_stop = e(max(1, n), torch.int64)
            self.total_frames = torch.zeros(1, dtype=torch.int64, device=dev)
        return self

    def to_struct(self) -> RhSegments:
        if self.buf.dtype != torch.uint8:
            raise ValueError("buf must be uint8")
        if self.seg_off.dtype != torch.int64 or self.seg_len.dtype != torch.int64:
            raise ValueError("seg_off and seg_len must be int64")
        if self.seg_len.numel() != self.n_seg:
            raise ValueError("seg_off and seg_len lengths differ")
        if self.scratch_off is None or self.scratch_off.numel() < self.n_seg * self.frames_per_seg_cap:
            raise ValueError("scratch too small for n_seg * frames_per_seg_cap (call alloc_outputs)")
        if self.frame_off.numel() < self.frame_cap or self.frame_len.numel() < self.frame_cap:
            raise ValueError("frame table smaller than frame_cap")
        g = RhSegments()
        g.buf = _ptr(self.buf)
        g.buf_len = self.buf.numel()
        g.seg_off = _ptr(self.seg_off)
        g.seg_len = _ptr(self.seg_len)
        g.n_seg = self.n_seg
        g.max_op = self.max_op
        g.frames_per_seg_cap = self.frames_per_seg_cap
        g.scratch_off = _ptr(self.scratch_off)
        g.scratch_len = _ptr(self.scratch_len)
        g.frame_off = _ptr(self.frame_off)
        g.frame_len = _ptr(self.frame_len)
        g.frame_cap = self.frame_cap
        g.seg_first = _ptr(self.seg_first)
        g.seg_nframes = _ptr(self.seg_nframes)
        g.seg_status = _ptr(self.seg_status)
        g.seg_stop = _ptr(self.seg_stop)
        g.total_frames = _ptr(self.total_frames)
        return g


def segments_scan(ctx: Context, batch: SegmentBatch, stream: Optional[torch.cuda.Stream] = None) -> None:
    """Enqueues the framing walk (asynchronous): fills the dense frame table and per-segment status."""
    batch.alloc_outputs()
    g = batch.to_struct()
    check(_lib.load().rh_segments_scan_launch(ctx.handle, ctypes.byref(g), _stream_ptr(stream)))


def read_segments(ctx: Context, batch: SegmentBatch, stream: Optional[torch.cuda.Stream] = None) -> dict:
    """``LogSegment.readSegmentFile`` over every segment: framing, then CRC32C verify of every frame,
    then each segment truncated at its first bad frame (``decodeEntry`` throws ChecksumException
    there, RDR:330-336).  Returns device tensors ``n_ok``, ``status``, ``stop`` per segment plus the
    frame table and CRC results.  All work stays on the device stream; tensor ops are glue only."""
    segments_scan(ctx, batch, stream)
    (stream or torch.cuda.current_stream()).synchronize()
    n_total = min(int(batch.total_frames.item()), batch.frame_cap)
    dev = batch.buf.device
    fb = FrameBatch(buf=batch.buf, frame_off=batch.frame_off[:n_total],
                    frame_len=batch.frame_len[:n_total]).alloc_outputs()
    if n_total:
        crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY, stream=stream)
    with torch.cuda.stream(stream) if stream is not None else _nullctx():
        nseg = batch.n_seg
        n_found = batch.seg_nframes[:nseg].to(torch.int64).clamp(max=batch.frames_per_seg_cap)
        first = batch.seg_first[:nseg]
        idx = torch.arange(n_total, device=dev)
        bad = ((fb.bad_bits.view(-1, 1) >> torch.arange(64, device=dev)) & 1).view(-1)[:n_total].bool()
        seg_of = torch.searchsorted(first, idx, right=True) - 1
        big = torch.iinfo(torch.int64).max
        first_bad = torch.full((nseg,), big, dtype=torch.int64, device=dev)
        first_bad.scatter_reduce_(0, seg_of[bad], idx[bad], reduce="amin")
        has_bad = first_bad < first + n_found
        n_ok = torch.where(has_bad, first_bad - first, n_found)
        status = torch.where(has_bad, torch.full_like(batch.seg_status[:nseg], RH_SEG_E_CHECKSUM),
                             batch.seg_status[:nseg])
        if n_total:
            stop_abs = batch.frame_off[first_bad.clamp(max=n_total - 1)]
            stop = torch.where(has_bad, stop_abs - batch.seg_off, batch.seg_stop[:nseg])
        else:
            stop = batch.seg_stop[:nseg].clone()
    return {"n_ok": n_ok, "status": status, "stop": stop, "frames": fb, "total_frames": batch.total_frames}


def read_segments_fused(ctx: Context, batch: SegmentBatch, stream: Optional[torch.cuda.Stream] = None) -> dict:
    """``LogSegment.readSegmentFile`` over every segment in one call (rh_segments_read_launch): the
    framing walk, every frame's CRC32C verify and the reader's verdict.  Fills the batch's framing
    outputs exactly as :func:`segments_scan` does and returns the reader's verdict per segment
    (``n_ok``, ``status``, ``stop``: the same values :func:`read_segments` derives) plus the dense
    per-frame CRCs / mismatch bits.  Asynchronous: nothing is synchronised."""
    batch.alloc_outputs()
    dev, n, cap = batch.buf.device, batch.n_seg, batch.frames_per_seg_cap
    out = {
        "scratch_crc": torch.empty(max(1, n * cap), dtype=torch.int32, device=dev),
        "n_ok": torch.empty(max(1, n), dtype=torch.int32, device=dev),
        "status": torch.empty(max(1, n), dtype=torch.int32, device=dev),
        "stop": torch.empty(max(1, n), dtype=torch.int64, device=dev),
        "crc_out": torch.empty(batch.frame_cap, dtype=torch.int32, device=dev),
        "bad_bits": torch.zeros((batch.frame_cap + 63) // 64, dtype=torch.int64, device=dev),
        "n_bad": torch.zeros(1, dtype=torch.int64, device=dev),
    }
    c = RhSegmentsCrc()
    c.scratch_crc = _ptr(out["scratch_crc"])
    c.seg_ok = _ptr(out["n_ok"])
    c.seg_read_status = _ptr(out["status"])
    c.seg_read_stop = _ptr(out["stop"])
    c.crc_out = _ptr(out["crc_out"])
    c.bad_bits = _ptr(out["bad_bits"])
    c.n_bad = _ptr(out["n_bad"])
    g = batch.to_struct()
    check(_lib.load().rh_segments_read_launch(ctx.handle, ctypes.byref(g), ctypes.byref(c), _stream_ptr(stream)))
    out["total_frames"] = batch.total_frames
    return out


def read_segments_host(ctx: Context, image, seg_off, seg_len, max_op: int = 4 << 20, frames_per_seg_cap: int = 4096,
                       frame_cap: Optional[int] = None) -> dict:
    """``rh_segments_read_host``: LogSegment.readSegmentFile's framing + checksum verdict for every
    segment of a HOST image (numpy uint8), PCIe included -- the call the Java module's bulk segment
    load makes.  Returns numpy arrays: per segment ``status``, ``n_ok``, ``stop``, ``first_frame``,
    ``n_frames``; per frame ``frame_off`` (in ``image``), ``frame_len``, ``frame_crc``; ``total``."""
    import numpy as np
    lib = _lib.load()
    img = np.ascontiguousarray(image, dtype=np.uint8)
    so = np.ascontiguousarray(seg_off, dtype=np.uint64)
    sl = np.ascontiguousarray(seg_len, dtype=np.uint64)
    n = so.size
    cap = n * frames_per_seg_cap if frame_cap is None else int(frame_cap)
    fo = np.zeros(max(cap, 1), dtype=np.uint64)
    fl = np.zeros(max(cap, 1), dtype=np.uint32)
    fc = np.zeros(max(cap, 1), dtype=np.uint32)
    res = (_lib.RhSegmentResult * max(n, 1))()
    total = ctypes.c_uint64()
    vp = ctypes.c_void_p
    check(lib.rh_segments_read_host(ctx.handle, vp(img.ctypes.data), img.size, vp(so.ctypes.data), vp(sl.ctypes.data),
                                    n, max_op, frames_per_seg_cap, vp(fo.ctypes.data), vp(fl.ctypes.data),
                                    vp(fc.ctypes.data), cap, res, ctypes.byref(total)))
    k = min(total.value, cap)
    return {"status": np.array([r.status for r in res[:n]], dtype=np.int32),
            "n_ok": np.array([r.n_ok for r in res[:n]], dtype=np.int64),
            "stop": np.array([r.stop for r in res[:n]], dtype=np.int64),
            "first_frame": np.array([r.first_frame for r in res[:n]], dtype=np.int64),
            "n_frames": np.array([r.n_frames for r in res[:n]], dtype=np.int64),
            "frame_off": fo[:k].astype(np.int64), "frame_len": fl[:k].astype(np.int64), "frame_crc": fc[:k],
            "total": int(total.value)}


def stamp_host(ctx: Context, buf, frame_off, frame_len) -> None:
    """``rh_crc32c_stamp_host``: every frame's 4-byte trailer in the HOST buffer ``buf`` (numpy uint8,
    modified in place) overwritten with the big-endian PureJavaCrc32C of the bytes before it --
    SegmentedRaftLogOutputStream.write's trailers (OUT:86-110) for a whole flush batch, PCIe
    included."""
    import numpy as np
    lib = _lib.load()
    assert isinstance(buf, np.ndarray) and buf.dtype == np.uint8 and buf.flags["C_CONTIGUOUS"]
    off = np.ascontiguousarray(frame_off, dtype=np.uint64)
    ln = np.ascontiguousarray(frame_len, dtype=np.uint32)
    vp = ctypes.c_void_p
    check(lib.rh_crc32c_stamp_host(ctx.handle, vp(buf.ctypes.data), buf.size, vp(off.ctypes.data),
                                   vp(ln.ctypes.data), off.size))


def pcie_write_probe(ctx: Context, nbytes: int = 64 << 20, reps: int = 9) -> float:
    """``rh_pcie_write_probe``: GB/s of GPU stores into mapped pinned host memory (the path the
    table's event records take), median of ``reps`` launches moving ``nbytes``."""
    ms = ctypes.c_float()
    check(_lib.load().rh_pcie_write_probe(ctx.handle, int(nbytes), int(reps), ctypes.byref(ms)))
    return nbytes / (ms.value * 1e-3) / 1e9


class HostRegistration:
    """``rh_host_register`` / ``rh_host_unregister`` of a numpy buffer (a context manager)."""

    def __init__(self, ctx: Context, buf):
        self._ctx, self._buf = ctx, buf
        check(_lib.load().rh_host_register(ctx.handle, ctypes.c_void_p(buf.ctypes.data), buf.nbytes))

    def close(self) -> None:
        if self._buf is not None:
            check(_lib.load().rh_host_unregister(self._ctx.handle, ctypes.c_void_p(self._buf.ctypes.data)))
            self._buf = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


# ---- leader lease ------------------------------------------------------------------------------
@dataclass
class LeaseTier:
    """Groups with the same follower-slot count F (0..14) for rh_lease_soa_launch."""

    follower_ts: torch.Tensor        # int64 [F, >=n] (column k = follower slot k), nanoTime values
    conf: torch.Tensor               # int32 [n] membership words
    lease_in: torch.Tensor           # int64 [n]
    enabled_bits: Optional[torch.Tensor] = None   # int64 [ceil(n/64)] or None (all enabled)
    lease_out: Optional[torch.Tensor] = None      # int64 [n]; may be lease_in itself
    has_lease_bits: Optional[torch.Tensor] = None  # int64 [ceil(n/64)]
    extended_bits: Optional[torch.Tensor] = None   # int64 [ceil(n/64)]

    @property
    def n(self) -> int:
        return int(self.conf.numel())

    def alloc_outputs(self, extended: bool = True) -> "LeaseTier":
        dev, nw = self.conf.device, (self.n + 63) // 64
        if self.lease_out is None:
            self.lease_out = torch.empty(self.n, dtype=torch.int64, device=dev)
        if self.has_lease_bits is None:
            self.has_lease_bits = torch.zeros(max(nw, 1), dtype=torch.int64, device=dev)
        if extended and self.extended_bits is None:
            self.extended_bits = torch.zeros(max(nw, 1), dtype=torch.int64, device=dev)
        return self

    def to_struct(self, now_nanos: int, timeout_ms: int) -> RhLeaseSoa:
        F = int(self.follower_ts.shape[0]) if self.follower_ts.dim() == 2 else 0
        if self.follower_ts.dtype != torch.int64 or self.lease_in.dtype != torch.int64:
            raise ValueError("follower_ts and lease_in must be int64")
        if F and self.follower_ts.stride(1) != 1 and self.n > 1:
            raise ValueError("follower_ts rows must be contiguous")
        if self.lease_in.numel() != self.n:
            raise ValueError("lease_in and conf lengths differ")
        t = RhLeaseSoa()
        t.n = self.n
        t.n_followers = F
        t.now_nanos = now_nanos
        t.timeout_ms = timeout_ms
        t.follower_ts = _ptr(self.follower_ts) if F else None
        t.col_stride = int(self.follower_ts.stride(0)) if F else self.n
        t.conf = _ptr(self.conf)
        t.lease_in = _ptr(self.lease_in)
        t.enabled_bits = _ptr(self.enabled_bits)
        t.lease_out = _ptr(self.lease_out)
        t.has_lease_bits = _ptr(self.has_lease_bits)
        t.extended_bits = _ptr(self.extended_bits)
        return t


@dataclass
class TiledLeaseTier:
    """A lease tier in the TILED layout of ``rh_lease_soa.tile_stride``: one int64 HBM buffer of
    ceil(n / 128) tiles, each holding for its 128 groups the F follower timestamp columns,
    lease_in and lease_out (128 int64 each), then the 128 uint32 membership words -- one
    contiguous run per tile for a wave's loads.  Bit columns stay plain."""

    n: int
    n_followers: int
    buf: torch.Tensor                # int64 [n_tiles, tile_elems]
    enabled_bits: Optional[torch.Tensor] = None
    has_lease_bits: Optional[torch.Tensor] = None
    extended_bits: Optional[torch.Tensor] = None

    @staticmethod
    def columns(F: int) -> List[str]:
        return [f"ts{k}" for k in range(F)] + ["lease_in", "lease_out"]

    @classmethod
    def from_arrays(cls, follower_ts, conf, lease_in, device="cuda", extended: bool = True) -> "TiledLeaseTier":
        import numpy as np
        F = int(follower_ts.shape[0]) if follower_ts.ndim == 2 else 0
        n = int(conf.size)
        nt = (n + 127) // 128
        cols = cls.columns(F)
        te = len(cols) * 128 + 64
        host = np.zeros((nt, te), dtype=np.int64)

        def put(name, a):
            c = cols.index(name)
            pad = np.zeros(nt * 128, dtype=np.int64)
            pad[:n] = a
            host[:, c * 128:(c + 1) * 128] = pad.reshape(nt, 128)
        for k in range(F):
            put(f"ts{k}", follower_ts[k])
        put("lease_in", lease_in)
        cw = np.zeros(nt * 128, dtype=np.uint32)
        cw[:n] = np.asarray(conf).view(np.uint32)
        host[:, len(cols) * 128:] = cw.reshape(nt, 128).view(np.int64)
        nw = max((n + 63) // 64, 1)
        t = cls(n=n, n_followers=F, buf=torch.from_numpy(host).to(device),
                has_lease_bits=torch.zeros(nw, dtype=torch.int64, device=device))
        if extended:
            t.extended_bits = torch.zeros(nw, dtype=torch.int64, device=device)
        return t

    def column(self, name: str) -> torch.Tensor:
        """Column ``name`` over the n groups (a gathered copy)."""
        c = self.columns(self.n_followers).index(name)
        return self.buf[:, c * 128:(c + 1) * 128].reshape(-1)[:self.n]

    @property
    def lease_out(self) -> torch.Tensor:
        return self.column("lease_out")

    def to_struct(self, now_nanos: int, timeout_ms: int) -> RhLeaseSoa:
        cols = self.columns(self.n_followers)
        base = self.buf.data_ptr()
        t = RhLeaseSoa()
        t.n = self.n
        t.n_followers = self.n_followers
        t.now_nanos = now_nanos
        t.timeout_ms = timeout_ms
        t.follower_ts = base if self.n_followers else None
        t.col_stride = 128
        t.conf = base + len(cols) * 128 * 8
        t.lease_in = base + cols.index("lease_in") * 128 * 8
        t.enabled_bits = _ptr(self.enabled_bits)
        t.lease_out = base + cols.index("lease_out") * 128 * 8
        t.has_lease_bits = _ptr(self.has_lease_bits)
        t.extended_bits = _ptr(self.extended_bits)
        t.tile_stride = int(self.buf.shape[1]) * 8
        return t


def lease_launch(ctx: Context, tiers: Sequence[LeaseTier], now_nanos: int, timeout_ms: int,
                 stream: Optional[torch.cuda.Stream] = None) -> None:
    """Enqueues the lease kernel for every tier (asynchronous)."""
    arr = (RhLeaseSoa * len(tiers))(*[t.to_struct(now_nanos, timeout_ms) for t in tiers])
    check(_lib.load().rh_lease_soa_launch(ctx.handle, arr, len(tiers), _stream_ptr(stream)))


def prepare_lease(tiers: Sequence, now_nanos: int, timeout_ms: int) -> PreparedLaunch:
    """lease_launch with the argument array built once."""
    return PreparedLaunch("rh_lease_soa_launch",
                          (RhLeaseSoa * len(tiers))(*[t.to_struct(now_nanos, timeout_ms) for t in tiers]), len(tiers))


def prepare_leader(commit_tiers: Sequence, lease_tiers: Sequence, now_nanos: int, timeout_ms: int) -> PreparedLaunch:
    """leader_launch with the argument arrays built once."""
    if not 1 <= len(commit_tiers) <= _lib.RH_MAX_TIERS or not 1 <= len(lease_tiers) <= _lib.RH_MAX_TIERS:
        raise ValueError("1..4 tiers of each kind per launch")
    c = (RhCommitSoa * len(commit_tiers))(*[t.to_struct(RH_MODE_COMMIT) for t in commit_tiers])
    ls = (RhLeaseSoa * len(lease_tiers))(*[t.to_struct(now_nanos, timeout_ms) for t in lease_tiers])
    return PreparedLaunch("rh_leader_soa_launch", c, len(commit_tiers), ls, len(lease_tiers))


def leader_launch(ctx: Context, commit_tiers: Sequence[CommitTier], lease_tiers: Sequence[LeaseTier], now_nanos: int,
                  timeout_ms: int, stream: Optional[torch.cuda.Stream] = None) -> None:
    """One fused launch: updateCommit over ``commit_tiers`` (COMMIT mode) and hasLease over
    ``lease_tiers`` (rh_leader_soa_launch; asynchronous)."""
    if not 1 <= len(commit_tiers) <= _lib.RH_MAX_TIERS or not 1 <= len(lease_tiers) <= _lib.RH_MAX_TIERS:
        raise ValueError("1..4 tiers of each kind per launch")
    c = (RhCommitSoa * len(commit_tiers))(*[t.to_struct(RH_MODE_COMMIT) for t in commit_tiers])
    ls = (RhLeaseSoa * len(lease_tiers))(*[t.to_struct(now_nanos, timeout_ms) for t in lease_tiers])
    check(_lib.load().rh_leader_soa_launch(ctx.handle, c, len(commit_tiers), ls, len(lease_tiers), _stream_ptr(stream)))
