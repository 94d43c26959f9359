"""Stage timing of the PCIe-inclusive commit path (bench.py's delta-streaming leg) on one GPU.

    python scripts/pcie_bench.py [--groups 1000000] [--steps 20] [--threads 16]

Prints JSON lines: the raw pinned H2D / D2H copy rates for one step's 16 MB of deltas (the bound
the pipelined path is measured against), then bench.delta_streaming's own figures.  Run under
`rocprofv3 --kernel-trace --memory-copy-trace --stats` for the per-stage device durations."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch

    import bench
    from ratis_amd import engine, workload
    ctx = engine.Context(0)
    nbytes = 16 * a.groups
    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    s = torch.cuda.Stream()
    for name, fn in (("h2d", lambda: d.copy_(h, non_blocking=True)), ("d2h", lambda: h.copy_(d, non_blocking=True))):
        with torch.cuda.stream(s):
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                fn()
            e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(json.dumps({"copy": name, "bytes": nbytes, "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)}))
    del h, d
    host = workload.commit_snapshot(a.groups, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    print(json.dumps({"delta_streaming": bench.delta_streaming(ctx, host, steps=a.steps, fill_threads=a.threads)}))


if __name__ == "__main__":
    main()
