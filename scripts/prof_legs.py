"""Per-leg kernel durations of a profiled bench.py run (tuning / evidence only).

    rocprofv3 --kernel-trace --marker-trace -d OUT -o run --output-format csv -- python3 bench.py ... > bench.log
    python scripts/prof_legs.py OUT bench.log > legs.md     (also writes OUT/legs.json)

bench.py opens a roctx range "leg:<name>" around every timed leg (bench._Legs).  Each kernel dispatch
of the trace is attributed to the range that holds its start; per leg and kernel the dispatch count
and the median / mean / min / max duration are listed, plus the leg's busy time per step (the sum of
its kernels' durations / steps, the spin kernel excluded) beside the figure the bench line derived
from HIP events for that leg -- the check that every roofline in the line can be recomputed from the
trace.
"""
import csv
import glob
import json
import os
import statistics
import sys

GATE = "spin_kernel"   # torch.cuda._sleep: the queue gate in front of each timed leg


# the kernel each roofline of the bench line prices (legs without an entry: every kernel of the step)
ROOFLINE_KERNEL = [("commit", "commit_kernel_rank"), ("lease", "lease_kernel"), ("fused", "leader_kernel"),
                   ("table_", "table_commit_kernel|table_list_kernel"), ("twatch_", "table_commit_kernel|table_list_kernel"),
                   ("crc", "crc_frames_kernel")]


def rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def marker_ranges(d):
    out = []
    for p in glob.glob(os.path.join(d, "**", "*marker_api_trace.csv"), recursive=True):
        for r in rows(p):
            name = next((v for v in r.values() if isinstance(v, str) and v.startswith("leg:")), None)
            if name:
                nm, _, k = name[4:].partition("#")
                out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), nm, int(k or 1)))
    return sorted(out)


def kernels(d):
    out = []
    for p in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in rows(p):
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    return sorted(out)


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0].strip()


def bench_figures(line):
    """The per-step ms the bench line reports for each leg, and where it sits in the line."""
    f = {}
    g = lambda *ks: _get(line, ks)  # noqa: E731
    f["commit"] = (g("roofline", "avg_launch_ms"), "roofline.avg_launch_ms")
    f["lease"] = (g("lease", "ms_per_pass"), "lease.ms_per_pass")
    f["fused"] = (g("lease", "fused_with_commit", "roofline", "avg_launch_ms"), "lease.fused_with_commit.roofline.avg_launch_ms")
    tc = g("pcie", "delta_streaming", "table_commit") or {}
    for k, v in tc.items():
        if isinstance(v, dict) and "auto" in v:
            leg = "table_" + k[len("dirty_"):] + "_auto"
            f[leg] = (v["auto"]["ms_evaluation"], f"pcie.delta_streaming.table_commit.{k}.auto.ms_evaluation")
    tw = g("pcie", "delta_streaming", "table_watch") or {}
    for k, v in tw.items():
        if isinstance(v, dict) and "ms_evaluation" in v:
            f["twatch_" + k[len("dirty_"):]] = (v["ms_evaluation"], f"pcie.delta_streaming.table_watch.{k}.ms_evaluation")
    f["crc"] = (g("crc32c", "roofline", "avg_launch_ms"), "crc32c.roofline.avg_launch_ms")
    f["framing"] = (g("crc32c", "read_path", "ms_framing"), "crc32c.read_path.ms_framing")
    f["framing_plus_verify"] = (g("crc32c", "read_path", "ms_framing_plus_verify"), "crc32c.read_path.ms_framing_plus_verify")
    f["read_launch"] = (g("crc32c", "read_path", "ms_read_launch"), "crc32c.read_path.ms_read_launch")
    f["ragged_framing"] = (g("crc32c", "read_path", "ragged", "ms_framing"), "crc32c.read_path.ragged.ms_framing")
    f["ragged_read_launch"] = (g("crc32c", "read_path", "ragged", "ms_read_launch"), "crc32c.read_path.ragged.ms_read_launch")
    return {k: v for k, v in f.items() if v[0] is not None}


def _get(d, ks):
    for k in ks:
        if not isinstance(d, dict) or k not in d:
            return None
        d = d[k]
    return d


def main():
    d = sys.argv[1]
    line = None
    if len(sys.argv) > 2:
        for ln in open(sys.argv[2]):
            ln = ln.strip()
            if ln.startswith("{") and '"metric"' in ln:
                line = json.loads(ln)
    rng = marker_ranges(d)
    ks = kernels(d)
    legs = {}
    for s, e, nm, k in rng:
        leg = legs.setdefault(nm, {"ranges": 0, "steps": 0, "kernels": {}})
        leg["ranges"] += 1
        leg["steps"] += k
        for ks_, ke, kn in ks:
            if s <= ks_ <= e:
                leg["kernels"].setdefault(short(kn), []).append((ke - ks_) / 1e3)
    figs = bench_figures(line) if line else {}
    out = {}
    print("| leg | kernel | dispatches | median us | mean us | min us | max us |")
    print("|---|---|---|---|---|---|---|")
    for nm in sorted(legs):
        leg = legs[nm]
        o = {"ranges": leg["ranges"], "steps": leg["steps"], "kernels": {}}
        busy = 0.0
        for kn, v in sorted(leg["kernels"].items(), key=lambda kv: -sum(kv[1])):
            st = {"n": len(v), "median_us": round(statistics.median(v), 2), "mean_us": round(statistics.mean(v), 2),
                  "min_us": round(min(v), 2), "max_us": round(max(v), 2)}
            o["kernels"][kn] = st
            if GATE not in kn:
                busy += sum(v)
            print(f"| {nm} | `{kn}` | {st['n']} | {st['median_us']} | {st['mean_us']} | {st['min_us']} | {st['max_us']} |")
        n_steps = leg["steps"]
        o["busy_us_per_step"] = round(busy / n_steps, 2) if n_steps else None
        main = [kn for kn in o["kernels"] if GATE not in kn]
        pick = next((sub for pre, sub in ROOFLINE_KERNEL if nm.startswith(pre)), None)
        if pick:   # the leg's roofline kernel
            main = [kn for kn in main if any(p in kn for p in pick.split("|"))] or main
        if main:   # else the kernel with the largest total time
            o["main_kernel"] = main[0]
            o["main_median_us"] = o["kernels"][main[0]]["median_us"]
        if nm in figs:
            o["bench_ms"], o["bench_field"] = figs[nm]
            if o["busy_us_per_step"]:
                o["trace_vs_bench"] = round(o["busy_us_per_step"] / (o["bench_ms"] * 1e3), 4)
            if o.get("main_median_us"):
                o["main_median_vs_bench"] = round(o["main_median_us"] / (o["bench_ms"] * 1e3), 4)
        out[nm] = o
    print()
    print("| leg | kernel busy us per step (trace) | main kernel median us | bench line us | busy / bench | "
          "main median / bench | bench field |")
    print("|---|---|---|---|---|---|---|")
    for nm, o in sorted(out.items()):
        if "bench_ms" in o:
            print(f"| {nm} | {o['busy_us_per_step']} | {o.get('main_median_us')} (`{o.get('main_kernel')}`) | "
                  f"{round(o['bench_ms'] * 1e3, 2)} | {o.get('trace_vs_bench')} | {o.get('main_median_vs_bench')} | "
                  f"`{o['bench_field']}` |")
    json.dump(out, open(os.path.join(d, "legs.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
