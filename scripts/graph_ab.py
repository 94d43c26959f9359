"""A/B: back-to-back stream launches vs one HIP graph replay of the same launches (commit and
lease kernels at config 3), to size the per-launch gap.  Tuning only.

    python scripts/graph_ab.py"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ratis_amd import _lib, engine, workload
    ctx = engine.Context(0)
    host = workload.commit_snapshot(1_000_000)
    R, K = 8, 64
    batches = []
    for r in range(R):
        tiers = []
        for h in host:
            t = workload.to_device(h)
            t.follower_index += r << 44
            t.self_index += r << 44
            t.commit_in += r << 44
            t.term_start += r << 44
            tiers.append(t.alloc_outputs())
        batches.append(tiers)
    s = torch.cuda.Stream()
    torch.cuda.synchronize()

    def stream_run(fn):
        with torch.cuda.stream(s):
            for i in range(8):
                fn(i)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for i in range(K):
                fn(i)
            e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / K * 1e3

    def graph_run(fn):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            for i in range(8):
                fn(i)
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            for i in range(K):
                fn(i)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(s):
            e0.record(s)
            g.replay()
            e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / K * 1e3

    commit = lambda i: engine.commit_launch(ctx, batches[i % R], stream=s)  # noqa: E731
    tiny = [workload.to_device(workload.stable_tier(1024)).alloc_outputs()]
    commit_tiny = lambda i: engine.commit_launch(ctx, tiny, stream=s)  # noqa: E731
    for name, fn in (("commit_1M", commit), ("commit_1k", commit_tiny)):
        for rep in range(3):
            print(json.dumps({"kernel": name, "rep": rep, "stream_us": round(stream_run(fn), 2),
                              "graph_us": round(graph_run(fn), 2)}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
