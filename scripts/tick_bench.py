"""A pump tick's latency on the resident table: push k follower replies (matchIndex / commitIndex
MAX deltas for k random divisions of config 3's 1M), then updateCommit and commitIndexChanged
(rh_commit_batch_async / _wait, rh_watch_levels_async / _wait) -- the host's wall clock from the
push to the last wait, median of `reps` ticks.  RATIS_HIP_LIB selects an A/B build.

    python scripts/tick_bench.py [--ks 256,2048,16384] [--reps 50]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--groups", type=int, default=1_000_000)
    ap.add_argument("--ks", type=str, default="256,2048,16384")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    from ratis_amd import _lib, engine, groups, workload
    ctx = engine.Context(0)
    host = workload.commit_snapshot(a.groups, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    n = sum(h.n for h in host)
    tab = groups.RaftGroupTable(ctx, capacity=n)
    first = 0
    for h in host:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        first += h.n
    tab.commit_wait_counts(tab.commit_async(watch_all=True))
    tab.watch_async()
    tab.watch_wait_count()
    match = np.concatenate([h.follower[:4] for h in host], axis=1)
    rng = np.random.default_rng(5)
    out = {}
    for k in (int(x) for x in a.ks.split(",")):
        ms = []
        for r in range(a.reps + 3):
            slot = rng.choice(n, size=k // 2, replace=False)
            col = rng.integers(0, 4, size=slot.size)
            match[col, slot] += rng.integers(1, 300, size=slot.size)
            d = groups.make_deltas(np.concatenate([slot, slot]), np.concatenate([col, 16 + col]),
                                   np.concatenate([match[col, slot], match[col, slot] - 2]))
            t0 = time.perf_counter()
            tab.push(d)
            tk = tab.commit_async(watch_all=True)
            tab.commit_wait_counts(tk)
            tab.watch_async()
            tab.watch_wait_count()
            if r >= 3:
                ms.append((time.perf_counter() - t0) * 1e3)
        out[f"k{k}"] = {"ms_tick_median": round(float(np.median(ms)), 4), "ms_tick_p90": round(float(np.percentile(ms, 90)), 4)}
    print(json.dumps({"lib": os.environ.get("RATIS_HIP_LIB", "default"), "ticks": out}))
    tab.close()


if __name__ == "__main__":
    main()
