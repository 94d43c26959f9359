"""Commit kernel sensitivity (tuning only): the config-3 launch in the tiled layout with and without
the bit columns and the min_out column, 8 rotating batches, median of 5 rounds."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from ratis_amd import engine, workload
    ctx = engine.Context(0)
    host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    alg = sum(h.algorithmic_bytes() for h in host)
    for name, kw in (("tiled", {}), ("tiled_joint_first", {"rev": True}), ("tiled_no_bits", {"bits": False}),
                     ("tiled_no_min", {"min": False}), ("tiled_no_bits_no_min", {"bits": False, "min": False}),
                     ("stable_only", {"only": 0}), ("joint_only", {"only": 1})):
        batches = []
        for r in range(8):
            tiers = []
            for h in host:
                d = r << 44
                t = engine.TiledCommitTier.from_arrays(h.follower + d, h.flush + d, h.conf, h.commit + d,
                                                       h.term_start + d, bits=kw.get("bits", True))
                t.min_out = kw.get("min", True)
                tiers.append(t)
            if kw.get("rev"):
                tiers = tiers[::-1]
            if "only" in kw:
                tiers = [tiers[kw["only"]]]
            batches.append(tiers)
        xs = []
        for _ in range(5):
            for i in range(8):
                engine.commit_launch(ctx, batches[i])
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for i in range(80):
                engine.commit_launch(ctx, batches[i % 8])
            e1.record()
            torch.cuda.synchronize()
            xs.append(e0.elapsed_time(e1) / 80 * 1e3)
        us = float(np.median(xs))
        a = alg if "only" not in kw else host[kw["only"]].algorithmic_bytes()
        print(json.dumps({"variant": name, "us_per_launch": round(us, 2), "alg_TBps": round(a / us / 1e6, 3)}), flush=True)
        del batches


if __name__ == "__main__":
    main()
