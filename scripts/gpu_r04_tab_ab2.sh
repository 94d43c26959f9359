# Round 4: tile evaluation A/B (non-temporal column loads; 8-wave workgroups) against the shipped
# build, alternating, the table leg at 100 / 10 % (kernel-boundary timing events).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04ab2}
mkdir -p $O && export TMPDIR=/tmp
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_nt.so ratis_amd/lib/ab/libratis_hip_w8.so ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_nt.so ratis_amd/lib/ab/libratis_hip_w8.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$R/$lib timeout -k 10 200 python -u scripts/table_bench.py --reps 10 --fracs 1.0,0.1 > $O/tb_$tag.log 2>&1 || { tail -20 $O/tb_$tag.log; exit 1; }
  python - $O/tb_$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
print(sys.argv[2], {k: (v["auto"]["ms_evaluation"], v["device"]["ms_evaluation"], v["sinks_agree"]) for k, v in d.items() if isinstance(v, dict)})
PY
done
