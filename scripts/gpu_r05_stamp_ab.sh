# Round 5: rh_crc32c_stamp_host per flush size (scripts/stamp_bench.py), the default library and the
# A/B builds under ratis_amd/lib/ab/, alternating, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05sa}
mkdir -p $O && export TMPDIR=/tmp
cd $R
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $(ls $R/ratis_amd/lib/ab/*.so 2>/dev/null); do
  tag=$(basename $lib .so)_$r
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/stamp_bench.py > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 - $O/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["write_stamp"]
print(sys.argv[2], "gpu_us", d["gpu_us"], "cpu_us", d["cpu_1core_us"], "crossover", d["crossover_bytes"], "parity", d["parity_ok"])
PY
done
done
