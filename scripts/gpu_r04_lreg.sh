# Round 4: list evaluation with region-major dealing (8 head regions, tier-tagged entries) -- table
# tests (list / tile interleaving, sinks, node, pump, JNI), then the table leg at 1 / 0.1 % under a
# kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04lr}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_pump.py tests/test_gpu_jni.py tests/test_gpu_table_lease.py tests/test_reference_sequences.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 6 --fracs 0.01,0.001 > $O/tb.log 2>&1 || { tail -20 $O/tb.log; exit 1; }
cd $R && python3 - $O/prof <<'PY'
import csv, sys
v = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000 for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv"))
     if "table_list_kernel" in r["Kernel_Name"]]
h = len(v) // 2
a, b = sorted(v[:h]), sorted(v[h:])
print("list kernel median 1 %:", round(a[len(a) // 2], 1) if a else None, " 0.1 %:", round(b[len(b) // 2], 1) if b else None, "n", len(v))
PY
