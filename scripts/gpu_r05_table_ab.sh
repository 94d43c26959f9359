# Round 5: resident-table evaluation A/B builds (RATIS_HIP_LIB, alternating, 2 rounds): the AUTO
# sink's evaluation time per dirty fraction (kernel-boundary HIP events, bench.table_commit_leg).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05t}
mkdir -p $O && export TMPDIR=/tmp
cd $R
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $(ls $R/ratis_amd/lib/ab/*.so 2>/dev/null); do
  tag=$(basename $lib .so)_$r
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/table_bench.py --reps 8 --fracs ${FRACS:-1.0,0.1,0.01} > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 - $O/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
print(sys.argv[2], {k: (round(v["auto"]["ms_evaluation"] * 1e3, 2), round(v["device"]["ms_evaluation"] * 1e3, 2), v["sinks_agree"])
                    for k, v in d.items() if isinstance(v, dict) and "auto" in v})
PY
done
done
