"""Fused read path (rh_segments_read_launch) tuning: timing + per-phase cycle breakdown.

    python scripts/readpath_bench.py [--segments 256] [--frame 4096] [--iters 5]
Prints JSON lines: GB/s of segment bytes for the two-pass path (framing, then CRC verify) and the
fused kernel, then the instrumented kernel's per-block cycle counters averaged over blocks."""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=256)
    ap.add_argument("--segment-size", type=int, default=32 << 20)
    ap.add_argument("--frame", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--variants", default="", help="comma list of fused-read variants to time")
    a = ap.parse_args()
    import torch

    from ratis_amd import _lib, engine, workload
    lib = _lib.load()
    ctx = engine.Context(0)
    ss = workload.synth_segments(ctx, n_segments=a.segments, segment_size=a.segment_size, frame_size=a.frame,
                                 corrupt_rate=0)
    n = ss.n_segments
    seg_bytes = n * ss.segment_size

    def batch():
        return engine.SegmentBatch(buf=ss.batch.buf,
                                   seg_off=torch.arange(n, device="cuda", dtype=torch.int64) * ss.segment_size,
                                   seg_len=torch.full((n,), ss.segment_size, device="cuda", dtype=torch.int64),
                                   frames_per_seg_cap=ss.frames_per_segment + 16)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    sb = batch()
    ms2 = timed(lambda: engine.read_segments(ctx, sb))
    ref = engine.read_segments(ctx, sb)
    torch.cuda.synchronize()
    ref_off = sb.frame_off[: int(sb.total_frames.item())].clone()
    print(json.dumps({"path": "two-pass", "shape": f"{n}x{ss.segment_size >> 20}MiB/{a.frame}B", "ms": round(ms2, 4),
                      "GBps": round(seg_bytes / (ms2 * 1e-3) / 1e9, 1)}), flush=True)
    variants = [int(v) for v in a.variants.split(",") if v] or [None]
    for v in variants:
        if v is not None:
            _lib.check(lib.rh_segments_read_set_variant(v))
        fb = batch()
        ms = timed(lambda: engine.read_segments_fused(ctx, fb))
        out = engine.read_segments_fused(ctx, fb)
        torch.cuda.synchronize()
        nf = int(fb.total_frames.item())
        ok = (nf == ref_off.numel() and torch.equal(fb.frame_off[:nf], ref_off)
              and torch.equal(out["n_ok"][:n].to(torch.int64).cpu(), ref["n_ok"][:n].to(torch.int64).cpu())
              and int(out["n_bad"].item()) == 0)
        # instrumented run
        _lib.check(lib.rh_segments_read_profile(1, None, 0))
        engine.read_segments_fused(ctx, fb)
        buf = (ctypes.c_uint64 * (1024 * 16))()
        _lib.check(lib.rh_segments_read_profile(0, ctypes.cast(buf, ctypes.c_void_p), 1024 * 16))
        pc = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 16)[: min(n, ctx_cus(torch))].astype(np.float64)
        m = pc.mean(axis=0)
        steps = max(m[4], 1)
        print(json.dumps({"path": "fused", "variant": v, "ms": round(ms, 4), "GBps": round(seg_bytes / (ms * 1e-3) / 1e9, 1),
                          "parity_vs_two_pass": bool(ok),
                          "cycles_per_step": {"total": round(m[0] / steps, 1), "walker_t0": round(m[1] / steps, 1),
                                              "fold_t64": round(m[2] / steps, 1), "t0_wait_end": round(m[3] / steps, 1),
                                              "t64_wait_start": round(m[5] / steps, 1),
                                              "t64_advance": round(m[8] / steps, 1), "fold_t1008": round(m[9] / steps, 1)},
                          "steps_per_block": round(steps, 1), "frames_per_step": round(m[6] / steps, 2),
                          "spec_frac": round(m[7] / max(m[6], 1), 3)}), flush=True)


def ctx_cus(torch):
    return torch.cuda.get_device_properties(0).multi_processor_count


if __name__ == "__main__":
    main()
