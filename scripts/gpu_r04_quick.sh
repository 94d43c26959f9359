# Round 4 quick loop: write-stamp leg + table leg (kernel trace) + the stamp/table GPU tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04k}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_write_stamp.py tests/test_gpu_table_events.py tests/test_gpu_crc.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u scripts/stamp_bench.py > $O/stamp.log 2>&1 || { tail -20 $O/stamp.log; exit 1; }
python - $O/stamp.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])["write_stamp"]
print("stamp", list(zip(d["sizes"], d["gpu_us"], d["cpu_1core_us"])), "crossover", d["crossover_bytes"], d["parity_ok"])
PY
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tprof -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 4 --fracs 1.0,0.1,0.01,0.001,0.0 > $O/tprof.log 2>&1 || { tail -20 $O/tprof.log; exit 1; }
cd $R && python - $O <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/tprof/**/*kernel_trace.csv", recursive=True)[0])))
for key in ("table_commit_kernel_rank<false>", "table_list_kernel<false>", "table_gather_kernel<false>"):
    print(key, [round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000, 1) for r in rows if key in r["Kernel_Name"]][-20:])
PY
