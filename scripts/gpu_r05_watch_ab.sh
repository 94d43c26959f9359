# Round 5: commitIndexChanged evaluation A/B (scripts/watch_bench.py per library, alternating, 2 rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05w}
mkdir -p $O && export TMPDIR=/tmp
cd $R
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $(ls $R/ratis_amd/lib/ab/*.so 2>/dev/null); do
  tag=$(basename $lib .so)_$r
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/watch_bench.py > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 - $O/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_watch"]
print(sys.argv[2], {k: (round(v["ms_evaluation"] * 1e3, 2), v["levels_changed"], v["sinks_agree"]) for k, v in d.items() if isinstance(v, dict)})
PY
done
done
