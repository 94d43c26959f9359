"""Minimal driver for rocprofv3 PMC passes: a few launches of one kernel configuration.

    python scripts/prof_kernels.py --what crc --segments 32 --iters 5
    python scripts/prof_kernels.py --what commit --iters 8
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["crc", "crcshape", "crcragged", "commit", "framing", "ragged", "ragged_read", "lease", "table"], default="crc")
    ap.add_argument("--max-frame", type=int, default=2048, help="ragged: frames of 64..max_frame bytes")
    ap.add_argument("--segments", type=int, default=32)
    ap.add_argument("--frame-size", type=int, default=516, help="crcshape: uniform frame size")
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch

    from ratis_amd import _lib, engine, workload
    ctx = engine.Context(0)
    if a.what == "framing":
        ss = workload.synth_segments(ctx, n_segments=a.segments, corrupt_rate=0)
        n = ss.n_segments
        sb = engine.SegmentBatch(buf=ss.batch.buf,
                                 seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * ss.segment_size,
                                 seg_len=torch.full((n,), ss.segment_size, device="cuda", dtype=torch.int64),
                                 frames_per_seg_cap=ss.frames_per_segment + 16)
        for _ in range(a.iters):
            engine.segments_scan(ctx, sb)
        torch.cuda.synchronize()
        print("seg_bytes", n * ss.segment_size, "segments", n)
    elif a.what == "ragged_read":
        rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=64, max_frame=a.max_frame, seed=7)
        n = rs.n_segments
        sb = engine.SegmentBatch(buf=rs.batch.buf,
                                 seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * rs.segment_size,
                                 seg_len=torch.full((n,), rs.segment_size, device="cuda", dtype=torch.int64),
                                 frames_per_seg_cap=int(rs.seg_nframes.max()) + 16)
        for _ in range(a.iters):
            engine.read_segments_fused(ctx, sb)
        torch.cuda.synchronize()
        print("seg_bytes", n * rs.segment_size, "segments", n)
    elif a.what == "ragged":
        rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=64, max_frame=a.max_frame, seed=7)
        n = rs.n_segments
        sb = engine.SegmentBatch(buf=rs.batch.buf,
                                 seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * rs.segment_size,
                                 seg_len=torch.full((n,), rs.segment_size, device="cuda", dtype=torch.int64),
                                 frames_per_seg_cap=int(rs.seg_nframes.max()) + 16)
        for _ in range(a.iters):
            engine.segments_scan(ctx, sb)
        torch.cuda.synchronize()
        print("seg_bytes", n * rs.segment_size, "segments", n)
    elif a.what == "table":
        # the resident table's updateCommit (table_commit_kernel_rank) with every row dirty, the
        # bench's table_commit 100 % step (bench.table_commit_leg): per row one delta, 10 % flush /
        # 90 % matchIndex of followers 0..3, +512 over the row's current value; RH_EVENTS_AUTO
        import numpy as np

        from ratis_amd import groups
        host = workload.commit_snapshot(1_000_000, seed=workload.SEED + 1)
        n = sum(h.n for h in host)
        tab = groups.RaftGroupTable(ctx, capacity=n)
        first = 0
        for h in host:
            tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
            first += h.n
        tab.commit_wait_counts(tab.commit_async(watch_all=True))
        cur_f = np.concatenate([h.follower[:4] for h in host], axis=1)
        cur_s = np.concatenate([h.flush for h in host])
        rng = np.random.default_rng(7)
        ev = []
        for i in range(a.iters):
            slot = rng.permutation(n)
            is_flush = rng.random(n) < 0.10
            col = rng.integers(0, 4, size=n)
            val = np.where(is_flush, cur_s[slot], cur_f[col, slot]) + 512
            cur_s[slot[is_flush]] = val[is_flush]
            cur_f[col[~is_flush], slot[~is_flush]] = val[~is_flush]
            tab.push(groups.make_deltas(slot, np.where(is_flush, _lib.RH_COL_FLUSH, col), val))
            ev.append(tab.commit_wait_counts(tab.commit_async(watch_all=True)))
        torch.cuda.synchronize()
        f_mean = (host[0].n * 4 + (n - host[0].n) * 6) / n
        na = sum(e[0] for e in ev) / len(ev)
        nw = sum(e[1] for e in ev) / len(ev)
        # bench.table_commit_leg's algorithmic bytes of a 100 % step (a tile evaluation into AUTO:
        # no records, 2 mask bits per row; mean over the iterations)
        alg = n * 1 + n * (8 * f_mean + 4 + 8 + 8 + 8 + 8 + 1) + na * (8 + 1) + nw * 8 + n / 4   # no row slots: REGION mode
        print("alg_bytes", int(alg), "rows", n, "advanced", int(na), "watch_all", int(nw))
    elif a.what == "lease":
        import numpy as np
        host = workload.commit_snapshot(1_000_000)
        rng = np.random.default_rng(3)
        now = 1 << 60
        batches = []
        for r in range(8):
            tiers = []
            for h in host:
                ts = now - rng.integers(0, 300_000_000, size=h.follower.shape, dtype=np.int64)
                lin = now - rng.integers(0, 200_000_000, size=h.n, dtype=np.int64)
                # the bench's default layout: tiled (rh_lease_soa.tile_stride)
                tiers.append(engine.TiledLeaseTier.from_arrays(ts, h.conf, lin))
            batches.append(tiers)
        torch.cuda.synchronize()
        for i in range(a.iters):
            engine.lease_launch(ctx, batches[i % 8], now, 100)
        torch.cuda.synchronize()
        alg = sum(h.follower.size * 8 + h.n * 20 + 2 * ((h.n + 63) // 64) * 8 for h in host)
        print("lease_bytes", alg, "groups", sum(h.n for h in host))
    elif a.what == "crcshape":
        ss = workload.synth_segments(ctx, n_segments=a.segments, frame_size=a.frame_size, corrupt_rate=0)
        for _ in range(a.iters):
            engine.crc32c_frames(ctx, ss.batch, flags=_lib.RH_CRC_VERIFY)
        torch.cuda.synchronize()
        print("frame_bytes", ss.frame_bytes, "frames", ss.batch.n)
    elif a.what == "crcragged":
        rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=64, max_frame=a.max_frame, seed=7)
        for _ in range(a.iters):
            engine.crc32c_frames(ctx, rs.batch, flags=_lib.RH_CRC_VERIFY)
        torch.cuda.synchronize()
        print("frames", rs.batch.n)
    elif a.what == "crc":
        ss = workload.synth_segments(ctx, n_segments=a.segments, corrupt_rate=0)
        for _ in range(a.iters):
            engine.crc32c_frames(ctx, ss.batch, flags=_lib.RH_CRC_VERIFY)
        torch.cuda.synchronize()
        print("frame_bytes", ss.frame_bytes, "frames", ss.batch.n)
    else:
        host = workload.commit_snapshot(1_000_000)
        batches = []
        for r in range(8):  # the bench's default layout: tiled (rh_commit_soa.tile_stride)
            d = r << 44
            batches.append([engine.TiledCommitTier.from_arrays(h.follower + d, h.flush + d, h.conf, h.commit + d,
                                                               h.term_start + d) for h in host])
        torch.cuda.synchronize()
        for i in range(a.iters):
            engine.commit_launch(ctx, batches[i % 8])
        torch.cuda.synchronize()
        print("alg_bytes", sum(h.algorithmic_bytes() for h in host), "groups", sum(h.n for h in host))
    ctx.close()


if __name__ == "__main__":
    main()
