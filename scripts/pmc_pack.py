"""Per-launch PMC counters of crc_pack_kernel from scripts/gpu_r03_pmcpack.sh passes.

    python scripts/pmc_pack.py gpurun_out/r03pk/pmc"""
import collections
import csv
import glob
import json
import sys


def main():
    d = sys.argv[1]
    out = {}
    for f in sorted(glob.glob(d + "/*/run_counter_collection.csv")):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "crc_pack_kernel" in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            out[k] = sum(v) / len(v)
    if "FETCH_SIZE" in out:
        out["hbm_read_bytes_corrected"] = out["FETCH_SIZE"] * 2 * 1024
    w = out.get("SQ_WAVES", 0) or 1
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
        if k in out:
            out[k + "_per_wave"] = out[k] / w
    print(json.dumps({k: round(v, 1) for k, v in out.items()}, indent=1))


if __name__ == "__main__":
    main()
