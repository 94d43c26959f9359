"""Per-kernel duration medians of the resident-table evaluation kernels in a rocprofv3 kernel trace
(tuning): python scripts/table_trace.py OUT/run_kernel_trace.csv"""
import collections
import csv
import statistics
import sys

d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
    n = n.split("(")[0]
    if n.startswith(("table_", "crc_")) or "commit_kernel" in n:
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    v = sorted(v)
    print(f"{k:45s} n={len(v):4d} median={statistics.median(v):8.2f} min={v[0]:8.2f} p25={v[len(v) // 4]:8.2f}")
