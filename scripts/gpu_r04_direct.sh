# Round 4: direct event lists (one range per workgroup, last workgroup publishes; no gather) -- the
# table / node / pump tests first, then the full GPU suite, the table leg at 100 / 10 / 1 / 0.1 %
# dirty, and a kernel trace of it.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04q}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_pump.py > $O/pytest_table.log 2>&1 || { tail -60 $O/pytest_table.log; exit 1; }
tail -1 $O/pytest_table.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u scripts/table_bench.py --fracs 1.0,0.1,0.01,0.001 > $O/tb.log 2>&1 || { tail -30 $O/tb.log; exit 1; }
python - $O/tb.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(k, "eval", v["ms_evaluation"], "list", v["list_mode"], "hm", v["host_mapped"], "dev", v["device"], "auto", v["auto"], "frac", v["roofline"]["frac"], "agree", v["sinks_agree"], "adv", v["advanced"])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 4 --fracs 1.0,0.1,0.01,0.001 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo prof done
