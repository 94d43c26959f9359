# Round 4: result-list D2H on its own stream (not behind the next deltas' H2D) -- table tests, then
# the PCIe legs (delta streaming, table leg) twice.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04d2h}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_pump.py tests/test_gpu_jni.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --crc-segments 0 --no-lease --no-cpu-baseline --steps 10 > $O/bench_$i.log 2>&1 || { tail -30 $O/bench_$i.log; exit 1; }
  python - $O/bench_$i.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
ds = d["pcie"]["delta_streaming"]
print("delta streaming ms/step", ds["ms_per_step"], ds.get("ms_per_step_runs"), ds.get("stage_ms"))
PY
done
