"""bench.table_watch_leg on its own (one GPU): commitIndexChanged over the resident table.

    python scripts/watch_bench.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from ratis_amd import engine, workload
    ctx = engine.Context(0)
    host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    print(json.dumps({"table_watch": bench.table_watch_leg(ctx, host)}))


if __name__ == "__main__":
    main()
