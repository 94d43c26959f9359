"""Where a sparse pump tick's host time goes (config 3's 1M groups, k replies): host clock per call
(push, rh_tick_async, the two waits), the empty tick (nothing marked: the launch + wait floor), and
with timing events the device split (submit = the staged deltas' apply, eval = the tick kernel).
One JSON line to stdout."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ratis_amd import engine, groups, workload  # noqa: E402

ctx = engine.Context(0)
host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED)
n_all = sum(h.n for h in host)
tab = groups.RaftGroupTable(ctx, capacity=n_all)
first = 0
for h in host:
    tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
    first += h.n
tab.commit_wait_counts(tab.tick_async())
tab.watch_wait_count()
match = np.concatenate([h.follower[:4] for h in host], axis=1)
rng = np.random.default_rng(9)


def deltas(k):
    slot = rng.choice(n_all, size=k // 2, replace=False)
    col = rng.integers(0, 4, size=slot.size)
    match[col, slot] += rng.integers(1, 300, size=slot.size)
    return groups.make_deltas(np.concatenate([slot, slot]), np.concatenate([col, 16 + col]),
                              np.concatenate([match[col, slot], match[col, slot] - 2]))


out = {}
for mode in ("tick_async", "two_calls"):
    for k in (0, 256, 2048):
        rows = []
        for r in range(110):
            d = deltas(k) if k else None
            t0 = time.perf_counter()
            if d is not None:
                tab.push(d)
            t1 = time.perf_counter()
            if mode == "tick_async":
                tk = tab.tick_async()
            else:
                tk = tab.commit_async()
                tab.watch_async()
            t2 = time.perf_counter()
            tab.commit_wait_counts(tk)
            t3 = time.perf_counter()
            tab.watch_wait_count()
            t4 = time.perf_counter()
            if r >= 10:
                rows.append((t1 - t0, t2 - t1, t3 - t2, t4 - t3, t4 - t0))
        a = np.median(np.array(rows), axis=0) * 1e6
        out[f"{mode}_k{k}_host_us"] = {"push": round(a[0], 1), "issue": round(a[1], 1), "wait_commit": round(a[2], 1),
                                       "wait_watch": round(a[3], 1), "total": round(a[4], 1)}
tab.set_timing(True)
for k in (0, 256, 2048):
    sp = []
    for r in range(60):
        if k:
            tab.push(deltas(k))
        tk = tab.tick_async()
        tab.commit_wait_counts(tk)
        tab.watch_wait_count()
        s = tab.last_timing_split()
        if r >= 10:
            sp.append((s["submit_ms"], s["eval_ms"], s["events_ms"], 2.0 if s["fused"] else 0.0))
    a = np.median(np.array(sp), axis=0) * 1e3
    out[f"tick_async_k{k}_device_us"] = {"submit": round(a[0], 1), "eval": round(a[1], 1), "events": round(a[2], 1),
                                         "fused": bool(a[3] > 1)}
tab.close()
ctx.close()
print(json.dumps(out), flush=True)
