"""rh_lease_batch over the resident table (the Java pump's hasLease pass, LeaderStateImpl.java:
1229-1249): config 3's 1M groups loaded, every lease enabled and every follower 0..3 stamped
recently, then `reps` passes timed with HIP events on the table stream (memset of the bitmap, the
lease kernels, the bitmap's D2H) and on the host (the whole call).  RATIS_HIP_LIB selects an A/B
build; run under rocprofv3 --kernel-trace for the kernel itself.

    python scripts/table_lease_bench.py [--groups 1000000] [--reps 20]"""
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
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    from ratis_amd import _lib, engine, groups, workload
    ctx = engine.Context(0)
    host = workload.commit_snapshot(a.groups, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    n = sum(h.n for h in host)
    tab = groups.RaftGroupTable(ctx, capacity=n)
    first = 0
    for h in host:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        first += h.n
    now = 10**15
    slots = np.arange(n, dtype=np.int64)
    tab.push_deltas(slots, _lib.RH_COL_LEASE_ON, np.ones(n, np.int64), ops=_lib.RH_OP_SET)
    tab.push_deltas(slots, _lib.RH_COL_LEASE, np.full(n, now - 10**9, np.int64), ops=_lib.RH_OP_SET)
    for k in range(4):
        tab.push_deltas(slots, _lib.RH_COL_TS(k), np.full(n, now - 1000 * (k + 1), np.int64), ops=_lib.RH_OP_SET)
    bits = tab.lease_batch(now, 1000)   # warm-up; applies the deltas
    stream = torch.cuda.ExternalStream(_lib.load().rh_ctx_stream(ctx.handle))
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    dev_ms, host_ms = [], []
    for r in range(a.reps):
        t = now + 1000 * (r + 1)
        e0.record(stream)
        h0 = time.perf_counter()
        tab.lease_async(t, 1000)
        e1.record(stream)
        bits = tab.lease_wait()
        host_ms.append((time.perf_counter() - h0) * 1e3)
        torch.cuda.synchronize()
        dev_ms.append(e0.elapsed_time(e1))
    print(json.dumps({"lib": os.environ.get("RATIS_HIP_LIB", "default"), "groups": n, "has_lease": int(bits.sum()),
                      "ms_device_median": round(float(np.median(dev_ms)), 4),
                      "ms_call_median": round(float(np.median(host_ms)), 4)}))
    tab.close()


if __name__ == "__main__":
    main()
