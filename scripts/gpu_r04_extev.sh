# Round 4: evaluation timing events stamped at the kernel boundaries (hipExtLaunchKernel) -- table
# tests, then the table leg (100 / 10 / 1 %) plain and under a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04ev}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_pump.py tests/test_gpu_jni.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/table_bench.py --reps 8 > $O/tb.log 2>&1 || { tail -30 $O/tb.log; exit 1; }
python - $O/tb.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(k, "eval", v["ms_evaluation"], "list", v["list_mode"], "auto", v["auto"], "frac", v["roofline"]["frac"], "agree", v["sinks_agree"])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 4 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo prof done
