"""Median GB/s per (kernel, shape) and build from gpurun_out/ab/*.log (scripts/gpu_ab.sh)."""
import collections
import glob
import json
import sys


def main():
    d0 = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab"
    res = collections.defaultdict(dict)
    for f in sorted(glob.glob(d0 + "/*.log")):
        tag = f.split("/")[-1][:-4].replace("libratis_hip", "") or "_"
        for line in open(f):
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            if "median_GBps" in d:
                res[d["kernel"] + " " + d.get("shape", "")][tag] = d["median_GBps"]
    tags = sorted({t for v in res.values() for t in v})
    print("| shape | " + " | ".join(tags) + " |")
    print("|---|" + "---|" * len(tags))
    for k, v in res.items():
        print(f"| {k} | " + " | ".join(f"{v[t]:.0f}" if t in v else "" for t in tags) + " |")


if __name__ == "__main__":
    main()
