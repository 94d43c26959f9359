"""Multi-GPU placement of RaftGroups and the node-wide stats reduction.

Groups shard by ``RaftGroupId.hashCode() mod nGPU`` (RaftId.java:119-122 delegates to
``java.util.UUID.hashCode``: ``hilo = msb ^ lsb; (int)(hilo >> 32) ^ (int)hilo``), floor-mod so a
negative hash still maps to [0, n).  Groups are independent, so the hot path has no inter-GPU
traffic; the only collective is one all-reduce of a small stats vector (RCCL over xGMI when
the process group is ``nccl``, gloo on CPU for tests).
"""
from __future__ import annotations

import numpy as np


def java_uuid_hash(msb: np.ndarray, lsb: np.ndarray) -> np.ndarray:
    """java.util.UUID.hashCode() for arrays of (mostSigBits, leastSigBits) as int64."""
    hilo = np.asarray(msb, dtype=np.int64) ^ np.asarray(lsb, dtype=np.int64)
    hi = (hilo >> np.int64(32)).astype(np.int32)   # (int)(hilo >> 32)
    lo = hilo.astype(np.int32)                      # (int)hilo: low 32 bits, two's complement
    return hi ^ lo


def shard_of(msb: np.ndarray, lsb: np.ndarray, n_shards: int) -> np.ndarray:
    """Math.floorMod(uuid.hashCode(), n_shards)."""
    h = java_uuid_hash(msb, lsb).astype(np.int64)
    return np.mod(h, n_shards).astype(np.int64)


def random_group_ids(n: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """Seeded random (type-4 style) UUID bit pairs, as RaftGroupId.randomId() would draw."""
    rng = np.random.Generator(np.random.PCG64(seed))
    msb = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=n, dtype=np.int64, endpoint=True)
    lsb = rng.integers(np.iinfo(np.int64).min, np.iinfo(np.int64).max, size=n, dtype=np.int64, endpoint=True)
    return msb, lsb


STATS_FIELDS = ("groups_evaluated", "commits_advanced", "frames_verified", "bytes_verified", "crc_mismatches")


def allreduce_stats(stats: dict, device=None) -> dict:
    """Sums the stats dict over all ranks of the default process group (identity when not
    initialised).  On GPU ranks the vector lives in HBM and the all-reduce runs over RCCL."""
    import torch
    import torch.distributed as dist

    vec = torch.tensor([int(stats.get(k, 0)) for k in STATS_FIELDS], dtype=torch.int64,
                       device=device if device is not None else "cpu")
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(vec, op=dist.ReduceOp.SUM)
    out = dict(stats)
    for k, v in zip(STATS_FIELDS, vec.tolist()):
        out[k] = v
    return out
