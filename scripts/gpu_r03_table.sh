# Round 3: resident-table commit kernel -- parity (table + node tests), then the stage timing of
# the shipped build and the A/B variants, then a kernel trace of the shipped build.
set -o pipefail
mkdir -p gpurun_out/r03t && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_table_lease.py tests/test_reference_sequences.py tests/test_gpu_segread.py > gpurun_out/r03t/pytest.log 2>&1 || { tail -40 gpurun_out/r03t/pytest.log; exit 1; }
tail -3 gpurun_out/r03t/pytest.log
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/*.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$PWD/$lib timeout -k 10 200 python -u scripts/table_bench.py > gpurun_out/r03t/tb_$tag.log 2>&1 || { tail -20 gpurun_out/r03t/tb_$tag.log; exit 1; }
  echo "== $tag"; python - gpurun_out/r03t/tb_$tag.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(" ", k, "hbm", v["ms_events_in_hbm"], "host", v["ms_events_host_mapped"], "frac", v["roofline"]["frac"], "agree", v["sinks_agree"], "adv", v["advanced"])
PY
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r03t/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/table_bench.py --reps 4 > $GRAFT_REPO_ROOT/gpurun_out/r03t/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r03t/prof.log; exit 1; }
echo prof done
