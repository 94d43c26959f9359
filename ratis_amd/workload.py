"""Synthetic leader-bookkeeping workloads of BASELINE.json.

There is no Ratis cluster behind the benchmark (no network, and the reference is a JVM library):
the inputs are seeded synthetic snapshots with the shapes the reference sees -- follower
matchIndex columns, the leader's flushIndex / commitIndex / current-term start, and the
membership words of stable and joint-consensus confs.

Commit snapshot generator (per group, seed 0x5241544953 via numpy PCG64):
  base          ~ U[2^20, 2^40)
  matchIndex    = base - U[0, 4096) for caught-up followers; 1% of entries = -1 (fresh follower,
                  FollowerInfoImpl.java:42); joint-conf newcomers lag base - U[0, 65536)
  flushIndex    = base - U[0, 64)                        (leader's own log, self slot)
  lastCommitted = base - U[64, 8192)
  termStart     = lastCommitted + U[-256, 4096)          (both branches of the term check)
  stable conf   = self + 4 followers (P = 5); 0.5% of groups have one follower without a
                  FollowerInfo, 0.5% are inactive (not leader)
  joint conf    (10%): old = self + followers 0..3; new replaces 1 (80%) or 2 (20%) old
                  followers by newcomers in slots 4, 5 (union 6 or 7 voters); 1% of joint
                  groups have the leader outside the new conf; 0.1% have an old conf with no
                  voter but listeners (=> getMajorityMin is empty, LeaderStateImpl.java:976-978)
Stable groups live in an F=4 tier, joint groups in an F=6 tier (unused slots masked out).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List

import numpy as np

from ._lib import RH_CONF_ACTIVE, RH_CONF_OLD_SHIFT, RH_CONF_SELF, RH_CONF_SELF_OLD, RH_CONF_TRANSITIONAL

SEED = 0x5241544953


@dataclass
class HostTier:
    follower: np.ndarray     # int64 [F, n]
    flush: np.ndarray        # int64 [n]
    commit: np.ndarray       # int64 [n]
    term_start: np.ndarray   # int64 [n]
    conf: np.ndarray         # uint32 [n]
    voters_union: np.ndarray  # int32 [n]: |new U old| voters incl. self (for algorithmic bytes)

    @property
    def n(self) -> int:
        return int(self.flush.size)

    @property
    def n_followers(self) -> int:
        return int(self.follower.shape[0])

    def algorithmic_bytes(self) -> int:
        """per group 8*P_union + 36 bytes (index columns incl. self, lastCommitted,
        termStart, membership word, commit write, watch-min write).  Padding not counted."""
        return int(np.sum(8 * self.voters_union.astype(np.int64) + 36))


def _indices(rng, n, F, base, lag_hi, neg_frac=0.01):
    lag = rng.integers(0, lag_hi, size=(F, n), dtype=np.int64)
    m = base[None, :] - lag
    neg = rng.random(size=(F, n)) < neg_frac
    m[neg] = -1
    return m


def _leader_cols(rng, n, base):
    flush = base - rng.integers(0, 64, size=n, dtype=np.int64)
    commit = base - rng.integers(64, 8192, size=n, dtype=np.int64)
    tstart = commit + rng.integers(-256, 4096, size=n, dtype=np.int64)
    return flush, commit, tstart


def stable_tier(n: int, seed: int = SEED, peers: int = 5) -> HostTier:
    rng = np.random.Generator(np.random.PCG64(seed))
    F = peers - 1
    base = rng.integers(1 << 20, 1 << 40, size=n, dtype=np.int64)
    follower = _indices(rng, n, F, base, 4096)
    flush, commit, tstart = _leader_cols(rng, n, base)
    new_mask = np.full(n, (1 << F) - 1, dtype=np.uint32)
    missing = rng.random(n) < 0.005
    drop = rng.integers(0, F, size=n).astype(np.uint32)
    new_mask[missing] &= ~(np.uint32(1) << drop[missing])
    conf = new_mask | np.uint32(RH_CONF_SELF) | np.uint32(RH_CONF_ACTIVE)
    inactive = rng.random(n) < 0.005
    conf[inactive] &= np.uint32(~RH_CONF_ACTIVE & 0xFFFFFFFF)
    union = np.full(n, peers, dtype=np.int32)
    return HostTier(follower, flush, commit, tstart, conf.astype(np.uint32), union)


def joint_tier(n: int, seed: int = SEED + 1) -> HostTier:
    """Transitional (old+new) groups, F = 6 follower slots."""
    rng = np.random.Generator(np.random.PCG64(seed))
    F = 6
    base = rng.integers(1 << 20, 1 << 40, size=n, dtype=np.int64)
    follower = _indices(rng, n, F, base, 4096)
    # newcomers (slots 4, 5) are catching up
    follower[4:6] = base[None, :] - rng.integers(0, 65536, size=(2, n), dtype=np.int64)
    flush, commit, tstart = _leader_cols(rng, n, base)
    two = rng.random(n) < 0.2
    old_mask = np.full(n, 0b1111, dtype=np.uint32)
    r1 = rng.integers(0, 4, size=n).astype(np.uint32)
    r2 = (r1 + 1 + rng.integers(0, 3, size=n).astype(np.uint32)) % 4
    new_mask = old_mask & ~(np.uint32(1) << r1)
    new_mask |= np.uint32(1 << 4)
    new_mask[two] &= ~(np.uint32(1) << r2[two])
    new_mask[two] |= np.uint32(1 << 5)
    # unused slot 5 for single replacements: index -1 (never selected)
    follower[5, ~two] = -1
    include_self = rng.random(n) >= 0.01
    include_self_old = np.ones(n, dtype=bool)
    empty_old = rng.random(n) < 0.001
    old_mask[empty_old] = 0
    include_self_old[empty_old] = False
    conf = (new_mask | (include_self.astype(np.uint32) * np.uint32(RH_CONF_SELF))
            | np.uint32(RH_CONF_TRANSITIONAL) | (old_mask << np.uint32(RH_CONF_OLD_SHIFT))
            | (include_self_old.astype(np.uint32) * np.uint32(RH_CONF_SELF_OLD)) | np.uint32(RH_CONF_ACTIVE))
    union = np.where(two, 7, 6).astype(np.int32)
    return HostTier(follower, flush, commit, tstart, conf.astype(np.uint32), union)


def commit_snapshot(n_groups: int, joint_frac: float = 0.10, peers: int = 5, seed: int = SEED) -> List[HostTier]:
    """BASELINE config 2 (peers=3, joint_frac=0) / config 3 (peers=5, joint_frac=0.1)."""
    n_joint = int(round(n_groups * joint_frac))
    tiers = [stable_tier(n_groups - n_joint, seed=seed, peers=peers)]
    if n_joint:
        tiers.append(joint_tier(n_joint, seed=seed + 1))
    return tiers


def to_device(tier: HostTier, device="cuda", gap_threshold: int = -1):
    """HostTier -> engine.CommitTier (torch HBM tensors)."""
    import torch

    from .engine import CommitTier

    def t(a, dt=torch.int64):
        return torch.from_numpy(np.ascontiguousarray(a)).to(device=device, dtype=dt)

    return CommitTier(follower_index=t(tier.follower), self_index=t(tier.flush),
                      conf=t(tier.conf.view(np.int32), torch.int32), commit_in=t(tier.commit),
                      term_start=t(tier.term_start), gap_threshold=gap_threshold)


def to_device_tiled(tier: HostTier, device="cuda", gap_threshold: int = -1, levels: bool = False):
    """HostTier -> engine.TiledCommitTier (the AoSoA layout of rh_commit_soa.tile_stride)."""
    from .engine import TiledCommitTier
    return TiledCommitTier.from_arrays(tier.follower, tier.flush, tier.conf, tier.commit, tier.term_start,
                                       device=device, gap_threshold=gap_threshold, levels=levels)


# ------------------------------------------------------------------------------------------
# Config 5: SegmentedRaftLog segments of fixed-size frames, synthesized in HBM
# ------------------------------------------------------------------------------------------
@dataclass
class SegmentSet:
    batch: object            # engine.FrameBatch (buf, frame_off, frame_len, outputs)
    n_segments: int
    segment_size: int
    frames_per_segment: int
    frame_size: int
    corrupted: np.ndarray    # sorted frame numbers whose payload was bit-flipped after stamping
    prefix_len: np.ndarray   # int32 [n_frames]: varint + LogEntryProto header bytes per frame

    @property
    def frame_bytes(self) -> int:
        return int(self.batch.frame_off.numel()) * self.frame_size


def _varint_cols(v: np.ndarray, size: int) -> np.ndarray:
    cols = [((v >> (7 * i)) & 0x7F) | (0x80 if i < size - 1 else 0) for i in range(size)]
    return np.stack(cols, axis=1).astype(np.uint8)


def synth_segments(ctx, n_segments: int, segment_size: int = 32 << 20, frame_size: int = 4096,
                   seed: int = SEED, corrupt_rate: float = 1e-6, first_segment: int = 0, device="cuda") -> SegmentSet:
    """Builds ``n_segments`` closed segment images in HBM: header
    "RaftLog1", frames of exactly ``frame_size`` bytes = varint(n) + LogEntryProto{term, index,
    stateMachineLogEntry{logData = seeded random}} + CRC, zero padding to ``segment_size``.
    CRCs are stamped by the GPU write-side kernel (RH_CRC_STAMP); then ``corrupt_rate`` of the
    frames get one payload bit flipped so verification has mismatches to find."""
    import torch

    from . import engine, segment
    from ._lib import RH_CRC_STAMP

    fps = (segment_size - len(segment.HEADER)) // frame_size
    n_frames = n_segments * fps
    total = n_segments * segment_size
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    buf = torch.randint(0, 256, (total,), dtype=torch.uint8, device=device, generator=gen)
    segv = buf.view(n_segments, segment_size)
    segv[:, :8] = torch.tensor(list(segment.HEADER), dtype=torch.uint8, device=device)
    used = 8 + fps * frame_size
    if used < segment_size:
        segv[:, used:] = 0
    seg_idx = np.repeat(np.arange(n_segments, dtype=np.int64), fps)
    k = np.tile(np.arange(fps, dtype=np.int64), n_segments)
    off = (seg_idx * segment_size + 8 + k * frame_size).astype(np.int64)
    gseg = seg_idx + first_segment
    term = 1 + gseg // 64
    index = gseg * fps + k + 1
    n = frame_size - 4
    n -= segment.varint_size(n)
    assert segment.varint_size(n) + n + 4 == frame_size
    vs_t = np.vectorize(segment.varint_size, otypes=[np.int64])(np.unique(term))
    prefix_len = np.zeros(n_frames, dtype=np.int32)
    prefix_rows = np.zeros((n_frames, 32), dtype=np.uint8)
    vst = np.ones(n_frames, dtype=np.int64)
    for i in range(1, 10):
        vst += (term >= (1 << (7 * i))).astype(np.int64)
    vsi = np.ones(n_frames, dtype=np.int64)
    for i in range(1, 10):
        vsi += (index >= (1 << (7 * i))).astype(np.int64)
    del vs_t
    for a in np.unique(vst):
        for b in np.unique(vsi[vst == a]):
            sel = np.nonzero((vst == a) & (vsi == b))[0]
            # template prefix for this (term size, index size) class
            p0 = segment.fixed_size_entry_prefix(1 << (7 * (a - 1)), 1 << (7 * (b - 1)), n)
            full = segment.varint(n) + p0
            L = len(full)
            rows = np.frombuffer(full, dtype=np.uint8)[None, :].repeat(sel.size, axis=0)
            v0 = len(segment.varint(n))
            rows[:, v0 + 1:v0 + 1 + a] = _varint_cols(term[sel], int(a))
            rows[:, v0 + 2 + a:v0 + 2 + a + b] = _varint_cols(index[sel], int(b))
            prefix_rows[sel, :L] = rows
            prefix_len[sel] = L
    # scatter prefixes into the image
    maxp = int(prefix_len.max())
    pos = torch.from_numpy(off).to(device)[:, None] + torch.arange(maxp, device=device)[None, :]
    val = torch.from_numpy(prefix_rows[:, :maxp]).to(device)
    mask = torch.from_numpy(np.arange(maxp)[None, :] < prefix_len[:, None]).to(device)
    buf[pos[mask]] = val[mask]
    del pos, val, mask
    fb = engine.FrameBatch(buf=buf, frame_off=torch.from_numpy(off).to(device),
                           frame_len=torch.full((n_frames,), frame_size, dtype=torch.int32, device=device))
    fb.alloc_outputs()
    engine.crc32c_frames(ctx, fb, flags=RH_CRC_STAMP)
    rng = np.random.Generator(np.random.PCG64(seed + 7))
    bad = np.nonzero(rng.random(n_frames) < corrupt_rate)[0]
    if bad.size:
        where = off[bad] + prefix_len[bad] + rng.integers(0, frame_size - 4 - prefix_len[bad])
        w = torch.from_numpy(where).to(device)
        buf[w] = buf[w] ^ 1
    torch.cuda.synchronize()
    return SegmentSet(fb, n_segments, segment_size, fps, frame_size, np.sort(bad), prefix_len)


@dataclass
class RaggedSegmentSet:
    batch: object            # engine.FrameBatch over every frame of every segment
    n_segments: int
    segment_size: int
    seg_nframes: np.ndarray  # int64 [n_segments]
    corrupted: np.ndarray    # sorted global frame numbers with one payload bit flipped


def synth_ragged_segments(ctx, n_segments: int, segment_size: int = 32 << 20, min_frame: int = 64,
                          max_frame: int = 2048, seed: int = SEED, corrupt_rate: float = 0.0,
                          device="cuda") -> RaggedSegmentSet:
    """Closed segment images whose frames have seeded random lengths in [min_frame, max_frame]
    (a log of differently sized entries, unlike config 5's fixed 4 KiB): header "RaftLog1",
    frames varint(n) + n payload bytes + CRC (payload = seeded random bytes, not a parsed
    LogEntryProto: framing and CRC never look inside it), zero padding.  CRCs stamped by the GPU
    write-side kernel, then ``corrupt_rate`` of the frames get one payload bit flipped."""
    import torch

    from . import engine, segment
    from ._lib import RH_CRC_STAMP

    assert 6 <= min_frame <= max_frame <= (1 << 14)
    rng = np.random.Generator(np.random.PCG64(seed))
    offs, lens, counts = [], [], []
    def frame_len(nn):  # varint_size(n) + n + 4, n < 2^14 here
        return np.where(nn >= 128, 2, 1) + nn + 4

    for s in range(n_segments):
        cap = segment_size - 8
        nn = rng.integers(max(1, min_frame - 5), max(1, max_frame - 6) + 1, size=cap // min_frame + 1)
        fl = frame_len(nn)
        end = np.cumsum(fl)
        k = int(np.searchsorted(end, cap, side="right"))
        fl = fl[:k]
        start = 8 + np.concatenate([[0], np.cumsum(fl)[:-1]]) if k else np.zeros(0, np.int64)
        offs.append(s * segment_size + start)
        lens.append(fl)
        counts.append(k)
    off = np.concatenate(offs).astype(np.int64)
    fl = np.concatenate(lens).astype(np.int64)
    # n with varint_size(n) + n + 4 == fl (every fl above came from such an n)
    n = fl - 5
    two = n >= 128
    n = np.where(two, fl - 6, n)
    assert np.all((n >= 128) == two) and np.all(n >= 1) and np.all(frame_len(n) == fl)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed)
    buf = torch.randint(0, 256, (n_segments * segment_size,), dtype=torch.uint8, device=device, generator=gen)
    segv = buf.view(n_segments, segment_size)
    segv[:, :8] = torch.tensor(list(segment.HEADER), dtype=torch.uint8, device=device)
    ends = np.array([o[-1] + l[-1] if len(o) else s * segment_size + 8 for s, (o, l) in enumerate(zip(offs, lens))])
    for s in range(n_segments):
        segv[s, int(ends[s] - s * segment_size):] = 0
    b0 = np.where(two, (n & 0x7F) | 0x80, n).astype(np.uint8)
    b1 = (n >> 7).astype(np.uint8)
    o_t = torch.from_numpy(off).to(device)
    buf[o_t] = torch.from_numpy(b0).to(device)
    o2 = torch.from_numpy(off[two] + 1).to(device)
    buf[o2] = torch.from_numpy(b1[two]).to(device)
    fb = engine.FrameBatch(buf=buf, frame_off=o_t, frame_len=torch.from_numpy(fl.astype(np.int32)).to(device))
    fb.alloc_outputs()
    engine.crc32c_frames(ctx, fb, flags=RH_CRC_STAMP)
    bad = np.nonzero(rng.random(off.size) < corrupt_rate)[0]
    if bad.size:
        hdr = np.where(two[bad], 2, 1)
        where = off[bad] + hdr + rng.integers(0, n[bad])
        w = torch.from_numpy(where).to(device)
        buf[w] = buf[w] ^ 1
    torch.cuda.synchronize()
    return RaggedSegmentSet(fb, n_segments, segment_size, np.asarray(counts, np.int64), np.sort(bad))
