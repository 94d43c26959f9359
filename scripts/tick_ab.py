"""The pump tick alone (bench.tick_leg): rh_tick_async (one launch) against the two calls, config 3's
1M groups, k = 256 / 2048 / 8192 replies per tick.  One JSON line to stdout."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ratis_amd import engine, workload  # noqa: E402

ctx = engine.Context(0)
host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED)
print(json.dumps(bench.tick_leg(ctx, host, ks=(256, 2048, 8192), reps=100)), flush=True)
ctx.close()
