# Round 5: producer push path A/B (RATIS_HIP_LIB: the default library and ratis_amd/lib/ab/*.so),
# scripts/push_probe.py then the reply-mix leg (scripts/reply_mix.py), alternating, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05pa}
mkdir -p $O && export TMPDIR=/tmp
cd $R
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $(ls $R/ratis_amd/lib/ab/*.so 2>/dev/null); do
  tag=$(basename $lib .so)_$r
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/push_probe.py > $O/probe_$tag.log 2>&1 || { tail -20 $O/probe_$tag.log; exit 1; }
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/reply_mix.py > $O/rm_$tag.log 2>&1 || { tail -20 $O/rm_$tag.log; exit 1; }
  python3 - $O/probe_$tag.log $O/rm_$tag.log $tag <<'PY'
import json, sys
p = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
m = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
print(sys.argv[3], {k: v["ms"] for k, v in p.items()}, "reply_mix ms/step", m["ms_per_step"], "producers", m["ms_producers_per_step"], "parity", m["parity_ok"])
PY
done
done
