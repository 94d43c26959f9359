"""Timing of the shipped kernels in ONE process (repeated rounds), for tuning.

    python scripts/microbench.py [--segments 32] [--rounds 5]
Prints one JSON line per kernel/shape: median/min/max GB/s over the rounds."""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=32)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--warm-ms", type=float, default=60.0, help="untimed run of each kernel/shape before its rounds")
    ap.add_argument("--only", default="crc,framing,commit,lease", help="comma list of sections to run")
    a = ap.parse_args()
    import torch

    from ratis_amd import _lib, engine, workload
    ctx = engine.Context(0)
    # calibration: what plain torch streaming kernels reach on this device
    x = torch.empty(1 << 27, dtype=torch.int64, device="cuda").random_()
    y = torch.empty_like(x)
    for name, fn, nbytes in (("copy_1GiB", lambda: y.copy_(x), 2 * x.numel() * 8),
                             ("sum_1GiB", lambda: x.sum(), x.numel() * 8)):
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        print(json.dumps({"kernel": "calibration:" + name, "GBps": round(nbytes / (e0.elapsed_time(e1) / 10 * 1e-3) / 1e9, 1)}))
    del x, y
    only = set(a.only.split(","))

    def timed(fn, nbytes, iters):
        # run the kernel for --warm-ms first: launch times settle only after tens of ms of load
        # (clock / power transient, profiles/r02/crc_warmup/), whatever the launch size
        t0 = time.perf_counter()
        while True:
            fn()
            torch.cuda.synchronize()
            if (time.perf_counter() - t0) * 1e3 >= a.warm_ms:
                break
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(iters):
            fn(i)
        e1.record()
        torch.cuda.synchronize()
        return nbytes / (e0.elapsed_time(e1) / iters * 1e-3) / 1e9

    def report(kernel, xs, **kw):
        x = np.array(xs)
        print(json.dumps({"kernel": kernel, **kw, "median_GBps": round(float(np.median(x)), 1),
                          "min_GBps": round(float(x.min()), 1), "max_GBps": round(float(x.max()), 1)}), flush=True)

    if "crc" in only:
        ss = workload.synth_segments(ctx, n_segments=a.segments, corrupt_rate=0)
        fb = ss.batch
        xs = [timed(lambda i=0: engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY), ss.frame_bytes, a.iters)
              for _ in range(a.rounds)]
        assert int(fb.n_bad.item()) == 0
        report("crc32c", xs, segments=a.segments)
        del ss, fb
        torch.cuda.empty_cache()

    if "crcshape" in only:
        # CRC cost per frame vs frame length (dense frame tables): uniform sizes, then ragged
        for fsz in (256, 516, 772, 1028, 1284, 1540, 2052, 4096):
            ss = workload.synth_segments(ctx, n_segments=a.segments, frame_size=fsz, corrupt_rate=0)
            fb = ss.batch
            xs = [timed(lambda i=0: engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY), ss.frame_bytes, a.iters)
                  for _ in range(a.rounds)]
            assert int(fb.n_bad.item()) == 0
            report("crc32c", xs, shape=f"uniform {fsz}B", frames=fb.n,
                   ns_per_frame=round(ss.frame_bytes / float(np.median(xs)) / fb.n, 3))
            del ss, fb
            torch.cuda.empty_cache()
        for lo, hi in ((64, 2048), (64, 512), (1024, 4096)):
            rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=lo, max_frame=hi)
            fb = rs.batch
            nbytes = int(fb.frame_len.sum().item())
            xs = [timed(lambda i=0: engine.crc32c_frames(ctx, fb, flags=_lib.RH_CRC_VERIFY), nbytes, a.iters)
                  for _ in range(a.rounds)]
            assert int(fb.n_bad.item()) == 0
            report("crc32c", xs, shape=f"ragged {lo}-{hi}B", frames=fb.n,
                   ns_per_frame=round(nbytes / float(np.median(xs)) / fb.n, 3))
            del rs, fb
            torch.cuda.empty_cache()

    if "ragread" in only:
        # rh_segments_read_launch (framing + CRC verify + verdict) over ragged 64-2048 B segments
        rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=64, max_frame=2048)
        n = rs.n_segments
        sb = engine.SegmentBatch(buf=rs.batch.buf, seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * rs.segment_size,
                                 seg_len=torch.full((n,), rs.segment_size, device="cuda", dtype=torch.int64),
                                 frames_per_seg_cap=int(rs.seg_nframes.max()) + 16)
        xs = [timed(lambda i=0: engine.read_segments_fused(ctx, sb), n * rs.segment_size, a.iters) for _ in range(a.rounds)]
        report("read_launch", xs, shape="ragged 64-2048B", segments=n)
        del rs, sb
        torch.cuda.empty_cache()

    if "readc5" in only:
        # rh_segments_read_launch over config-5 segments (4 KiB frames)
        ss = workload.synth_segments(ctx, n_segments=a.segments, corrupt_rate=0)
        n = ss.n_segments
        sb = engine.SegmentBatch(buf=ss.batch.buf, seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * ss.segment_size,
                                 seg_len=torch.full((n,), ss.segment_size, device="cuda", dtype=torch.int64),
                                 frames_per_seg_cap=ss.frames_per_segment + 16)
        xs = [timed(lambda i=0: engine.read_segments_fused(ctx, sb), n * ss.segment_size, a.iters) for _ in range(a.rounds)]
        report("read_launch", xs, shape="config5 4096B", segments=n)
        del ss, sb
        torch.cuda.empty_cache()

    def framing(sets, tag):
        buf, n, seg_size, cap, nfr = sets
        sb = engine.SegmentBatch(buf=buf, seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * seg_size,
                                 seg_len=torch.full((n,), seg_size, device="cuda", dtype=torch.int64),
                                 frames_per_seg_cap=cap)
        xs = [timed(lambda i=0: engine.segments_scan(ctx, sb), n * seg_size, a.iters) for _ in range(a.rounds)]
        assert int(sb.total_frames.item()) == nfr
        report("segments_scan", xs, shape=tag, segments=n)

    if "framing" in only:
        for seg_size, fsz in ((32 << 20, 4096), (32 << 20, 512)):
            ss = workload.synth_segments(ctx, n_segments=a.segments, segment_size=seg_size, frame_size=fsz,
                                         corrupt_rate=0)
            framing((ss.batch.buf, ss.n_segments, ss.segment_size, ss.frames_per_segment + 16, ss.batch.n),
                    f"{seg_size >> 20}MiBx{fsz}B")
            del ss
            torch.cuda.empty_cache()
        for lo, hi in ((64, 2048), (64, 512)):
            rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=lo, max_frame=hi)
            framing((rs.batch.buf, rs.n_segments, rs.segment_size, int(rs.seg_nframes.max()) + 16,
                     int(rs.seg_nframes.sum())), f"32MiBx{lo}-{hi}B ragged")
            del rs
            torch.cuda.empty_cache()

    host = workload.commit_snapshot(1_000_000)
    if "commit" in only:
        alg = sum(h.algorithmic_bytes() for h in host)
        batches = []
        for r in range(8):
            tiers = []
            for h in host:
                t = workload.to_device(h)
                t.follower_index += r << 44
                t.self_index += r << 44
                t.commit_in += r << 44
                t.term_start += r << 44
                tiers.append(t.alloc_outputs())
            batches.append(tiers)
        xs = [timed(lambda i=0: engine.commit_launch(ctx, batches[i % 8]), alg, 40) for _ in range(a.rounds)]
        report("commit", xs, layout="plain", median_Gupd_s=round(float(np.median(xs)) * 1e9 / alg * 1e6 / 1e9, 2))
        del batches
        batches = [[engine.TiledCommitTier.from_arrays(h.follower + (r << 44), h.flush + (r << 44), h.conf,
                                                       h.commit + (r << 44), h.term_start + (r << 44)) for h in host]
                   for r in range(8)]
        xs = [timed(lambda i=0: engine.commit_launch(ctx, batches[i % 8]), alg, 40) for _ in range(a.rounds)]
        report("commit", xs, layout="tiled", median_Gupd_s=round(float(np.median(xs)) * 1e9 / alg * 1e6 / 1e9, 2))
        del batches
    if "lease" in only:
        now, ms, tmo = 1 << 60, 1_000_000, 100
        rng = np.random.default_rng(5)
        lb = []
        lalg = 0
        for r in range(8):
            tiers = []
            for h in host:
                ts = now - rng.integers(-ms, 3 * tmo * ms, size=h.follower.shape, dtype=np.int64)
                lin = now - rng.integers(0, 2 * tmo * ms, size=h.n, dtype=np.int64)
                if r == 0:
                    lalg += ts.size * 8 + h.n * 4 + h.n * 16 + 2 * ((h.n + 63) // 64) * 8
                t = engine.LeaseTier(follower_ts=torch.from_numpy(ts).cuda(),
                                     conf=torch.from_numpy(h.conf.view(np.int32)).cuda(),
                                     lease_in=torch.from_numpy(lin).cuda())
                tiers.append(t.alloc_outputs())
            lb.append(tiers)
        xs = [timed(lambda i=0: engine.lease_launch(ctx, lb[i % 8], now, tmo), lalg, 40) for _ in range(a.rounds)]
        report("lease", xs)
    ctx.close()


if __name__ == "__main__":
    main()
