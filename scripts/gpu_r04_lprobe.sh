# Round 4 probe: where the list evaluation's time goes (scan / list entry / rows / events), builds
# that stop after each stage (RH_LIST_PROBE, wrong results, timing only), 1 % and 0.1 % dirty.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04lp}
mkdir -p $O && export TMPDIR=/tmp
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_lw8.so ratis_amd/lib/ab/libratis_hip_lw16.so ratis_amd/lib/libratis_hip.so; do
  tag=$(basename $lib .so)
  cd /tmp && RATIS_HIP_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$tag -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 6 --fracs 0.01,0.001 > $O/tb_$tag.log 2>&1 || { tail -20 $O/tb_$tag.log; exit 1; }
  cd $R
  python3 - $O/prof_$tag $tag <<'PY'
import csv, sys
v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv"))
     if "table_list_kernel" in r["Kernel_Name"]]
h = len(v) // 2
a, b = sorted(v[:h]), sorted(v[h:])
print(sys.argv[2], "list kernel median 1 %:", round(a[len(a) // 2], 1) if a else None, " 0.1 %:", round(b[len(b) // 2], 1) if b else None, "n", len(v))
PY
done
