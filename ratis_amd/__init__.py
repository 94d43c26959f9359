"""ratis_amd -- MI355X-native leader-bookkeeping engine for Apache Ratis (OneSizeFitsQuorum/ratis).

Hot paths (BASELINE.json north_star): batched quorum commit (LeaderStateImpl.updateCommit /
getMajorityMin / RaftLogBase.updateCommitIndex) and SegmentedRaftLog CRC32C (PureJavaCrc32C),
as HIP kernels for gfx950 behind the C ABI of include/ratis_hip.h (lib/libratis_hip.so).

Modules:
  _lib      ctypes binding of the C ABI (fails loudly if the native library is missing)
  engine    device-side API over torch-owned HBM: Context, CommitTier, FrameBatch, launches
  groups    RaftGroupTable / RaftNode: the resident per-GPU table the Java ratis-hip module holds,
            and one RaftServer's tables over several GPUs
  segment   segment/frame layout and LogEntryProto encoding (host side)
  workload  seeded synthetic workloads of BASELINE.json
  shard     RaftGroupId placement across GPUs and the RCCL stats all-reduce
"""
__all__ = ["_lib", "engine", "groups", "segment", "workload", "shard"]
__version__ = "0.1.0"
