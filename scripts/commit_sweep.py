"""Headline kernel size sweep (tuning / evidence only): commit_kernel_rank over config-3-shaped
snapshots (5 peers, 10 % joint) of 2k .. 4M groups, tiled layout, rotating over enough distinct
batches that every launch streams HBM (>= 615 MB per rotation, like bench.py).  Per size: HIP-event
time per launch back to back (K launches behind a queue gate) and the algorithmic bytes, so the
time splits into a fixed part and a per-byte part (least squares over the sizes >= 0.25M).

    python scripts/commit_sweep.py [--sizes 2048,250000,...] [--launches 200]

Run under rocprofv3 --kernel-trace --marker-trace to get per-dispatch durations per size
(roctx ranges "leg:sweep_<n>#K", scripts/prof_legs.py).
"""
import argparse
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="2048,65536,250000,500000,1000000,2000000,4000000")
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--no-bits", action="store_true", help="ablation: no valid / advanced bit columns")
    ap.add_argument("--no-min", action="store_true", help="ablation: no min_out column")
    ap.add_argument("--tiers", choices=["both", "stable", "joint"], default="both", help="ablation: one tier only")
    a = ap.parse_args()
    import torch

    from bench import LEGS, queue_gate
    from ratis_amd import engine, workload
    ctx = engine.Context(0)
    stream = torch.cuda.current_stream()
    pts = []
    for n in [int(x) for x in a.sizes.split(",")]:
        host = workload.commit_snapshot(n, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
        if a.tiers != "both":
            host = [host[0 if a.tiers == "stable" else 1]]
        alg = sum(h.algorithmic_bytes() for h in host)
        R = max(8, math.ceil(615e6 / alg))
        batches = []
        for r in range(R):
            d = r << 44
            tiers = [engine.TiledCommitTier.from_arrays(h.follower + d, h.flush + d, h.conf, h.commit + d,
                                                        h.term_start + d, bits=not a.no_bits) for h in host]
            if a.no_min:
                for t in tiers:
                    t.min_out = False
            batches.append(tiers)
        launches = [engine.prepare_commit(b) for b in batches]
        for i in range(2 * R):
            launches[i % R](ctx, stream)
        torch.cuda.synchronize()
        xs = []
        for _ in range(a.rounds):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            LEGS.push(f"sweep_{n}", a.launches)
            queue_gate(stream)
            e0.record(stream)
            for i in range(a.launches):
                launches[i % R](ctx, stream)
            e1.record(stream)
            torch.cuda.synchronize()
            LEGS.pop()
            xs.append(e0.elapsed_time(e1) / a.launches * 1e3)
        us = float(np.median(xs))
        pts.append((n, alg, us))
        print(json.dumps({"groups": n, "rotating_batches": R, "alg_bytes": alg, "us_per_launch": round(us, 3),
                          "rounds_us": [round(x, 3) for x in xs], "alg_TBps": round(alg / us / 1e6, 3)}), flush=True)
        del batches, launches
        torch.cuda.empty_cache()
    fit = [(b, u) for n, b, u in pts if n >= 250_000]
    if len(fit) >= 2:
        A = np.array([[1.0, b / 1e6] for b, _ in fit])
        y = np.array([u for _, u in fit])
        (c0, c1), *_ = np.linalg.lstsq(A, y, rcond=None)
        print(json.dumps({"fit": "us = fixed + per_MB * MB (sizes >= 0.25M groups)", "fixed_us": round(float(c0), 3),
                          "per_MB_us": round(float(c1), 5), "marginal_TBps": round(1.0 / float(c1), 3)}), flush=True)


if __name__ == "__main__":
    main()
