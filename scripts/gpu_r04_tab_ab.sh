# Round 4: resident-table evaluation A/B (persistent grid, summary, no-events floor), table leg per
# build, then a kernel trace of every build's run.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04c
mkdir -p $O && export TMPDIR=/tmp
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/*.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$R/$lib timeout -k 10 200 python -u scripts/table_bench.py --reps 6 > $O/tb_$tag.log 2>&1 || { tail -20 $O/tb_$tag.log; exit 1; }
  echo "== $tag"; python - $O/tb_$tag.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(" ", k, "eval", v["ms_evaluation_kernel"], "gather_dev", v["device"]["ms_gather"], "agree", v["sinks_agree"], "adv", v["advanced"])
PY
done
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_persist512.so ratis_amd/lib/ab/libratis_hip_noev.so; do
  tag=$(basename $lib .so)
  cd /tmp && RATIS_HIP_LIB=$R/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$tag -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 4 > $O/prof_$tag.log 2>&1 || { tail -20 $O/prof_$tag.log; exit 1; }
  cd $R
done
echo done
