"""The bench's reply-mix delta leg alone (tuning): python scripts/reply_mix.py [--threads 16]."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    import bench
    from ratis_amd import workload
    host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    print(json.dumps(bench.reply_mix_leg(host, threads=a.threads, steps=a.steps)), flush=True)


if __name__ == "__main__":
    main()
