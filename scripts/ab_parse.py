"""Per-kernel average durations (us) of the kernel-trace runs an A/B script left under one
gpurun_out directory (one sub-directory per workload and library, e.g. ragged_read_libratis_hip_x3_2).

    python scripts/ab_parse.py gpurun_out/<tag> [kernel substrings ...]"""
import collections
import csv
import glob
import sys


def main():
    root = sys.argv[1]
    keys = sys.argv[2:] or ["crc_pack", "piece_guess", "piece_walk", "crc_frames"]
    res = collections.defaultdict(dict)
    for d in sorted(glob.glob(root + "/*_libratis_hip*")):
        g = glob.glob(d + "/**/run_kernel_stats.csv", recursive=True)
        if not g:
            continue
        tag = d.rstrip("/").split("/")[-1]
        for r in csv.DictReader(open(g[0])):
            n = r["Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            if any(k in n for k in keys):
                res[tag][n] = round(float(r["AverageNs"]) / 1000, 1)
    for t in sorted(res, key=lambda t: (t.split("_libratis")[0], t.rsplit("_", 1)[-1])):
        print(t, res[t])


if __name__ == "__main__":
    main()
