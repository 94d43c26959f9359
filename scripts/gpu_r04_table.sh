# Round 4: table v2 (tiled rows, tile summaries, per-XCD event heads + gather) -- full GPU suite,
# the table leg at 100 / 10 / 1 % dirty, and a kernel trace of it.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04i
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/table_bench.py > $O/tb.log 2>&1 || { tail -30 $O/tb.log; exit 1; }
python - $O/tb.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(k, "eval", v["ms_evaluation_kernel"], "hm", v["host_mapped"], "dev", v["device"], "frac", v["roofline"]["frac"], "agree", v["sinks_agree"], "adv", v["advanced"])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 4 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
echo prof done
cd $R && timeout -k 10 200 python -u scripts/stamp_bench.py > $O/stamp.log 2>&1 || { tail -20 $O/stamp.log; exit 1; }
tail -1 $O/stamp.log
