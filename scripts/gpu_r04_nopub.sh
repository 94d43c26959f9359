# Round 4 probe: what the last workgroup's host-mapped length write costs the tile evaluation
# (probe build skips it: wrong list lengths, timing only), 100 / 10 % dirty, alternating builds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04np}
mkdir -p $O && export TMPDIR=/tmp
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_nopub.so ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_nopub.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$R/$lib timeout -k 10 200 python -u scripts/table_bench.py --reps 10 --fracs 1.0,0.1 > $O/tb_$tag.log 2>&1 || { tail -20 $O/tb_$tag.log; exit 1; }
  python - $O/tb_$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
print(sys.argv[2], {k: (v["auto"]["ms_evaluation"], v["device"]["ms_evaluation"], v["host_mapped"]["ms_evaluation"]) for k, v in d.items() if isinstance(v, dict)})
PY
done
