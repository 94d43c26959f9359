"""bench.delta_streaming on its own (one GPU; RATIS_HIP_LIB selects an A/B build): 1M deltas per step
through the pinned ring, pipelined with the evaluations.  One JSON line to stdout."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from ratis_amd import engine, workload  # noqa: E402

ctx = engine.Context(0)
host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
r = bench.delta_streaming(ctx, host, fill_threads=bench.cpu_threads())
print(json.dumps({"lib": os.environ.get("RATIS_HIP_LIB", "default"), "delta_streaming": r}), flush=True)
