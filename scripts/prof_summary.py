"""Per-(kernel, grid) dispatch statistics from a rocprofv3 --kernel-trace CSV.

    python scripts/prof_summary.py gpurun_out/<tag>/prof/run_kernel_trace.csv [--out profiles/...md]

rocprofv3's --stats summary averages every dispatch of a kernel name; bench.py launches the hot
kernels with several shapes (the timed 1M-group batch, the PCIe sections, the group tables), so
this splits them by grid size.  The row whose grid matches the timed launch is the one to compare
with bench.py's roofline.avg_launch_ms (events over back-to-back launches, so bench's figure is
slightly larger: it includes the gaps between kernels)."""
import argparse
import collections
import csv
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default=None)
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    groups = collections.defaultdict(list)
    for r in csv.DictReader(open(a.trace)):
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
        if name.startswith("void "):
            name = name[5:]
        short = name.split("(")[0]
        short = short if len(short) <= 90 else short[:87] + "..."
        key = (short, int(r["Grid_Size_X"]), int(r["Workgroup_Size_X"]), int(r["VGPR_Count"]), int(r["LDS_Block_Size"]))
        groups[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    rows = sorted(groups.items(), key=lambda kv: -sum(kv[1]))[: a.top]
    lines = ["| kernel | grid (threads) | wg | VGPR | LDS B | calls | mean us | median us | min us | total ms |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    for (name, grid, wg, vgpr, lds), d in rows:
        lines.append(f"| `{name}` | {grid} | {wg} | {vgpr} | {lds} | {len(d)} | {statistics.mean(d):.2f} | "
                     f"{statistics.median(d):.2f} | {min(d):.2f} | {sum(d) / 1e3:.3f} |")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        open(a.out, "w").write(f"Source: `{a.trace}` (rocprofv3 --kernel-trace of `python3 bench.py`)\n\n" + txt + "\n")


if __name__ == "__main__":
    main()
