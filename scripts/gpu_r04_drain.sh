# Round 4: AUTO sink's tile evaluations drained into the pinned lists by a kernel on the side stream
# -- table / node / pump / JNI tests, delta streaming per sink, the table leg.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04dr}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_pump.py tests/test_gpu_jni.py tests/test_gpu_table_lease.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u scripts/ds_bench.py > $O/ds.log 2>&1 || { tail -30 $O/ds.log; exit 1; }
grep -v "^{" $O/ds.log | tail -4
timeout -k 10 300 python -u scripts/table_bench.py --reps 8 > $O/tb.log 2>&1 || { tail -30 $O/tb.log; exit 1; }
python - $O/tb.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(k, "eval", v["ms_evaluation"], "auto call", v["auto"]["ms_commit_batch_async_hip_events"], "frac", v["roofline"]["frac"], "agree", v["sinks_agree"])
PY
