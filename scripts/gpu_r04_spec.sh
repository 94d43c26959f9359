# Round 4: tile evaluation with the column loads issued beside the flag load (SPEC) against the
# summary-then-flags-then-columns build -- table tests, then the table leg (100 / 10 / 3 % dirty)
# under a kernel trace per build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04sp}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_pump.py tests/test_gpu_jni.py tests/test_gpu_table_lease.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in ratis_amd/lib/libratis_hip.so; do
  tag=$(basename $lib .so)
  cd /tmp && RATIS_HIP_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$tag -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 6 --fracs 1.0,0.1,0.04 > $O/tb_$tag.log 2>&1 || { tail -20 $O/tb_$tag.log; exit 1; }
  cd $R
  python3 - $O/prof_$tag $tag <<'PY'
import csv, sys
v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv"))
     if "table_commit_kernel_rank" in r["Kernel_Name"]]
# per case: 7 rounds x 3 sinks; keep device + auto (not host_mapped = every 3rd from index 0)
out = []
for c in range(3):
    seg = v[1 + c * 21: 1 + (c + 1) * 21]
    da = sorted(x for i, x in enumerate(seg) if i % 3 != 0)
    out.append(round(da[len(da) // 2], 1))
print(sys.argv[2], "median dev/auto us at 100/10/4 %:", out)
PY
done
