# Round 4: tile evaluation clipped to each tier's high-water mark -- table tests, the table leg,
# and the table PMC passes (FETCH / WRITE).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04hw}
mkdir -p $O/pmc && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_pump.py tests/test_gpu_table_lease.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/table_bench.py --reps 8 > $O/tb.log 2>&1 || { tail -30 $O/tb.log; exit 1; }
python - $O/tb.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(k, "eval", v["ms_evaluation"], "list", v["list_mode"], "frac", v["roofline"]["frac"], "agree", v["sinks_agree"])
PY
cd /tmp
run() { local name=$1 ctrs=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$O/pmc/$name" -o run --output-format csv -- python3 $R/scripts/prof_kernels.py "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run table_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what table --iters 6
run table_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what table --iters 6
run table_w "WRITE_SIZE" --what table --iters 6
echo done
