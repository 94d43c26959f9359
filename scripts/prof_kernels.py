"""Minimal driver for rocprofv3 PMC passes: a few launches of one kernel configuration.

    python scripts/prof_kernels.py --what crc --variant 0 --segments 32 --iters 5
    python scripts/prof_kernels.py --what commit --variant 0 --iters 8
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--what", choices=["crc", "commit"], default="crc")
    ap.add_argument("--variant", type=int, default=0)
    ap.add_argument("--segments", type=int, default=32)
    ap.add_argument("--iters", type=int, default=5)
    a = ap.parse_args()
    import torch

    from ratis_amd import _lib, engine, workload
    ctx = engine.Context(0)
    if a.what == "crc":
        ss = workload.synth_segments(ctx, n_segments=a.segments, corrupt_rate=0)
        for _ in range(a.iters):
            engine.crc32c_frames(ctx, ss.batch, flags=_lib.RH_CRC_VERIFY, variant=a.variant)
        torch.cuda.synchronize()
        print("frame_bytes", ss.frame_bytes, "frames", ss.batch.n)
    else:
        _lib.check(_lib.load().rh_commit_set_variant(a.variant))
        host = workload.commit_snapshot(1_000_000)
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
        torch.cuda.synchronize()
        for i in range(a.iters):
            engine.commit_launch(ctx, batches[i % 8])
        torch.cuda.synchronize()
        print("alg_bytes", sum(h.algorithmic_bytes() for h in host), "groups", sum(h.n for h in host))
    ctx.close()


if __name__ == "__main__":
    main()
