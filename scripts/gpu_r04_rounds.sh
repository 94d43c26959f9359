# Round 4 probe: is the 100 %-dirty tile evaluation paying a partial second round of workgroups?
# The table leg at 100 % for tables of 0.39M .. 1.57M groups under a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04r1}
mkdir -p $O && export TMPDIR=/tmp
for n in 393216 770000 1000000 1200000 1572864; do
  cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$n -o run --output-format csv -- python3 $R/scripts/table_bench.py --groups $n --reps 4 --fracs 1.0 > $O/tb_$n.log 2>&1 || { tail -20 $O/tb_$n.log; exit 1; }
  cd $R
done
python3 - $O <<'PY'
import csv, glob, os, re, sys
for d in sorted(glob.glob(sys.argv[1] + "/prof_*"), key=lambda p: int(p.rsplit("_", 1)[1])):
    v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(d + "/run_kernel_trace.csv"))
         if "table_commit_kernel_rank" in r["Kernel_Name"]]
    v = sorted(v)
    print(os.path.basename(d), "n", len(v), "min", round(v[0], 1), "median", round(v[len(v) // 2], 1))
PY
