"""The pump's tick over several shards on one GPU (HipLeaderBookkeeper.tick: every shard's
evaluations issued before any wait): 4 shards x 250k config-3 groups, k replies per shard per tick,
rh_tick_async against the two calls, ticks alternating.  Host clock from the first push to the last
wait; one JSON line to stdout."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ratis_amd import groups, workload  # noqa: E402

S, N = 4, 250_000
node = groups.RaftNode(0, N, devices=[0] * S)
mats = []
for s, t in enumerate(node.tables):
    host = workload.commit_snapshot(N, joint_frac=0.10, peers=5, seed=workload.SEED + s)
    first = 0
    for h in host:
        t.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        first += h.n
    mats.append((first, np.concatenate([h.follower[:4] for h in host], axis=1)))
    t.commit_wait_counts(t.tick_async())
    t.watch_wait_count()
rng = np.random.default_rng(3)
out = {}
for k in (256, 2048):
    ms = {"tick_async": [], "two_calls": []}
    for r in range(2 * 100 + 6):
        fused = r % 2 == 0
        ds = []
        for n_all, match in mats:
            slot = rng.choice(n_all, size=k // 2, replace=False)
            col = rng.integers(0, 4, size=slot.size)
            match[col, slot] += rng.integers(1, 300, size=slot.size)
            ds.append(groups.make_deltas(np.concatenate([slot, slot]), np.concatenate([col, 16 + col]),
                                         np.concatenate([match[col, slot], match[col, slot] - 2])))
        t0 = time.perf_counter()
        tks = []
        for t, d in zip(node.tables, ds):
            t.push(d)
        for t in node.tables:
            if fused:
                tks.append(t.tick_async())
            else:
                tks.append(t.commit_async())
                t.watch_async()
        for t, tk in zip(node.tables, tks):
            t.commit_wait_counts(tk)
            t.watch_wait_count()
        t1 = time.perf_counter()
        if r >= 6:
            ms["tick_async" if fused else "two_calls"].append((t1 - t0) * 1e6)
    out[f"replies_{k}_per_shard"] = {m: {"median_us": round(float(np.median(v)), 1),
                                         "p90_us": round(float(np.percentile(v, 90)), 1)} for m, v in ms.items()}
node.close()
out["workload"] = f"{S} shards x {N} config-3 groups on one GPU; per tick per shard k deltas; host clock, 100 ticks each"
print(json.dumps(out), flush=True)
