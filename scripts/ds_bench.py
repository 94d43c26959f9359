"""bench.delta_streaming on its own, per event sink (A/B): python scripts/ds_bench.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from ratis_amd import _lib, engine, workload
    ctx = engine.Context(0)
    host = workload.commit_snapshot(1_000_000, joint_frac=0.10, peers=5, seed=workload.SEED + 1)
    out = {}
    for name, sink in (("auto", _lib.RH_EVENTS_AUTO), ("host_mapped", _lib.RH_EVENTS_HOST_MAPPED),
                       ("device", _lib.RH_EVENTS_DEVICE), ("auto2", _lib.RH_EVENTS_AUTO)):
        r = bench.delta_streaming(ctx, host, fill_threads=bench.cpu_threads(), sink=sink)
        out[name] = {k: r[k] for k in ("ms_per_step", "ms_per_step_runs", "stage_ms")}
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
