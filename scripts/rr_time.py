"""Times rh_segments_read_launch on bench.py's ragged workload (256 x 32 MiB, 64-2048 B frames,
the bench's seed) with HIP events, for same-box A/B of library builds (RATIS_HIP_LIB).

    python scripts/rr_time.py [--segments 256] [--steps 10] [--rounds 3]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--segments", type=int, default=256)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    import torch

    from ratis_amd import engine, workload
    ctx = engine.Context()
    dev = torch.device("cuda")
    rs = workload.synth_ragged_segments(ctx, n_segments=a.segments, min_frame=64, max_frame=2048,
                                        seed=workload.SEED + 5, corrupt_rate=1e-5)
    n, size = rs.n_segments, rs.segment_size
    cap = int(rs.seg_nframes.max()) + 16
    fb = engine.SegmentBatch(buf=rs.batch.buf, seg_off=torch.arange(n, dtype=torch.int64, device=dev) * size,
                             seg_len=torch.full((n,), size, dtype=torch.int64, device=dev), frames_per_seg_cap=cap)
    s = torch.cuda.current_stream()
    for _ in range(2):
        engine.read_segments_fused(ctx, fb, stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = []
    for _ in range(a.rounds):
        torch.cuda.synchronize()
        e0.record(s)
        for _ in range(a.steps):
            engine.read_segments_fused(ctx, fb, stream=s)
        e1.record(s)
        torch.cuda.synchronize()
        out.append(round(e0.elapsed_time(e1) / a.steps, 4))
    print("read_launch_ms", out, "lib", os.path.basename(os.environ.get("RATIS_HIP_LIB", "libratis_hip.so")))
    ctx.close()


if __name__ == "__main__":
    main()
