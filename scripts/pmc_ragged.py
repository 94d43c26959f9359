"""HBM traffic of one ragged read launch (rh_segments_read_launch over 64-2048 B frames) from
rocprofv3 PMC passes of scripts/prof_kernels.py --what ragged_read (scripts/gpu_r03_final.sh):
FETCH_SIZE (x2, the gfx950 wide-read undercount, MI355X_MICROARCH.md) + WRITE_SIZE summed over
the library's kernels of the run, divided by the launches and by the segment bytes.

    python scripts/pmc_ragged.py gpurun_out/<tag>/pmc --iters 4 [--merge profiles/r03/pmc_traffic.json]"""
import argparse
import collections
import csv
import json
import os

OURS = ("crc_", "piece_", "segment_")


def sums(path):
    """Counters summed over the library's kernels dispatched from the first read-path kernel on
    (the synthetic images' CRC stamping runs before it and is not counted)."""
    rows = list(csv.DictReader(open(path)))
    first = min(int(r["Dispatch_Id"]) for r in rows if "segment_" in r["Kernel_Name"])
    tot = collections.defaultdict(float)
    pack = collections.defaultdict(float)
    for r in rows:
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        if not name.startswith(OURS) or int(r["Dispatch_Id"]) < first:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
        if name.startswith("crc_pack_kernel"):
            pack[r["Counter_Name"]] += float(r["Counter_Value"])
    return tot, pack


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_dir")
    ap.add_argument("--iters", type=int, required=True, help="read launches in the profiled run")
    ap.add_argument("--merge", default=None, help="pmc_traffic.json to add the figures to")
    a = ap.parse_args()
    fb, fp = sums(os.path.join(a.pmc_dir, "rr_b", "run_counter_collection.csv"))
    wb, wp = sums(os.path.join(a.pmc_dir, "rr_w", "run_counter_collection.csv"))
    seg = None
    for line in open(os.path.join(a.pmc_dir, "rr_b.log")):
        if line.startswith("seg_bytes"):
            seg = int(line.split()[1])
    n = a.iters
    fetch = fb["FETCH_SIZE"] * 2 * 1024 / n
    write = wb["WRITE_SIZE"] * 1024 / n
    out = {"ragged_read_fetch_bytes_per_launch": round(fetch), "ragged_read_write_bytes_per_launch": round(write),
           "ragged_read_bytes_per_launch": round(fetch + write), "ragged_read_units_per_launch": seg,
           "ragged_read_bytes_per_unit": round((fetch + write) / seg, 4),
           "ragged_pack_fetch_bytes_per_launch": round(fp["FETCH_SIZE"] * 2 * 1024 / n),
           "ragged_pack_write_bytes_per_launch": round(wp["WRITE_SIZE"] * 1024 / n)}
    print(json.dumps(out, indent=1))
    if a.merge:
        d = json.load(open(a.merge)) if os.path.exists(a.merge) else {}
        d.update(out)
        d["ragged_read_source"] = a.pmc_dir
        open(a.merge, "w").write(json.dumps(d, indent=1) + "\n")


if __name__ == "__main__":
    main()
