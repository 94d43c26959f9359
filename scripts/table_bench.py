"""bench.table_commit_leg on its own (one GPU): the resident table's rh_commit_batch at 100 % and
10 % dirty groups, events staged in HBM and host-mapped.  RATIS_HIP_LIB selects an A/B build.

    python scripts/table_bench.py [--groups 1000000] [--reps 8]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--fracs", type=str, default="1.0,0.1,0.01")
    a = ap.parse_args()
    import bench
    from ratis_amd import engine, workload
    ctx = engine.Context(0)
    host = workload.commit_snapshot(a.groups, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    r = bench.table_commit_leg(ctx, host, reps=a.reps, fracs=tuple(float(x) for x in a.fracs.split(",")))
    print(json.dumps({"lib": os.environ.get("RATIS_HIP_LIB", "default"), "table_commit": r}))


if __name__ == "__main__":
    main()
