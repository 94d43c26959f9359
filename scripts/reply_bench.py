"""bench.reply_mix_leg on its own (one GPU): 16 native producers push config 3's per-reply delta
mix through rh_node_push_deltas, the pump's evaluations pipelined behind.  RATIS_HIP_LIB selects
an A/B build.

    python scripts/reply_bench.py [--groups 1000000] [--runs 3]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--runs", type=int, default=3)
    a = ap.parse_args()
    import bench
    from ratis_amd import workload
    host = workload.commit_snapshot(a.groups, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    runs = [bench.reply_mix_leg(host, threads=bench.cpu_threads()) for _ in range(a.runs)]
    print(json.dumps({"lib": os.environ.get("RATIS_HIP_LIB", "default"),
                      "ms_per_step": [r["ms_per_step"] for r in runs],
                      "ms_producers_per_step": [r["ms_producers_per_step"] for r in runs],
                      "parity_ok": all(r["parity_ok"] for r in runs)}))


if __name__ == "__main__":
    main()
