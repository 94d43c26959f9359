"""Per-kernel averages of rocprofv3 --pmc CSVs: python scripts/pmc_table.py <dir-glob-prefix> [match]."""
import collections
import csv
import glob
import sys


def main():
    pre, match = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in sorted(glob.glob(pre + "*/run_counter_collection.csv")):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if match not in k:
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(k, " ".join(f"{c}={sum(x) / len(x):.4g}" for c, x in sorted(v.items())))


if __name__ == "__main__":
    main()
