"""Piece-walk latency vs concurrency: frame n ragged 32 MiB segments (64-2048 B) a few times; run
under rocprofv3 --kernel-trace --stats once per n and compare piece_walk_kernel's duration (the
walk is one dependent header load per frame, ~250 per 256 KiB piece, independent of n)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from ratis_amd import engine, workload

n = int(sys.argv[1])
ctx = engine.Context(0)
rs = workload.synth_ragged_segments(ctx, n, min_frame=64, max_frame=2048, seed=5)
size = rs.segment_size
b = engine.SegmentBatch(buf=rs.batch.buf, seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * size,
                        seg_len=torch.full((n,), size, device="cuda", dtype=torch.int64),
                        frames_per_seg_cap=int(rs.seg_nframes.max()) + 16)
for _ in range(5):
    engine.segments_scan(ctx, b)
torch.cuda.synchronize()
nf = int(rs.seg_nframes.sum())
assert int(b.total_frames.item()) == nf and torch.equal(b.frame_off[:nf], rs.batch.frame_off)
print("ok", n, nf)
