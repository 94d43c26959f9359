"""Where the multi-producer push time goes (tuning): rh_node_push_deltas from T native producer
threads (bench._producers) into one 1.1M-row table, no evaluations.  Per T: the time of a push of
0.9M deltas (fits the open staging slot: validation + copy only) and of 4M deltas (4 slots: the
slot hand-offs, each waiting for the H2D of the slot two fills back).

    python scripts/push_probe.py"""
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from ratis_amd import _lib, groups, workload
    lib = _lib.load()
    host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    n_all = sum(h.n for h in host)
    node = groups.RaftNode(0, n_all, devices=[0])
    tab = node.tables[0]
    first = 0
    for h in host:
        tab.load(first, h.conf, h.flush, h.commit, h.term_start, match=h.follower)
        first += h.n
    torch.cuda.synchronize()
    rng = np.random.default_rng(3)
    push_fn = ctypes.cast(lib.rh_node_push_deltas, ctypes.c_void_p).value
    out = {}
    for T in (1, 4, 8, 16):
        prod = bench._producers(T)
        T = prod.threads()
        for n in (900_000, 4_000_000):
            slot = np.sort(rng.integers(0, n_all, n)).astype(np.uint32)
            d = groups.make_deltas(slot, rng.integers(0, 4, n), rng.integers(0, 1 << 40, n))
            shares = np.linspace(0, n, T + 1).astype(np.uint64)
            xs = []
            for r in range(4):
                tab.commit_wait_counts(tab.commit_async(watch_all=False))   # drain the staged deltas
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                if prod.push(push_fn, node._h.value, d.ctypes.data, shares.ctypes.data, 4096) != 0:
                    raise RuntimeError("push failed")
                xs.append(time.perf_counter() - t0)
            out[f"T{T}_n{n}"] = {"ms": round(float(np.median(xs[1:])) * 1e3, 3),
                                 "ns_per_delta_per_thread": round(float(np.median(xs[1:])) / n * T * 1e9, 1)}
            print(f"T{T}_n{n}", out[f"T{T}_n{n}"], flush=True)
        prod.close()
    node.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
