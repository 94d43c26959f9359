# Round 5: commit / lease / fused kernel A/B builds: bench.py without the CRC, ragged, PCIe and CPU
# legs, per library (RATIS_HIP_LIB), alternating, 2 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05l}
mkdir -p $O && export TMPDIR=/tmp
cd $R
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $(ls $R/ratis_amd/lib/ab/*.so 2>/dev/null); do
  tag=$(basename $lib .so)_$r
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u bench.py --crc-segments 0 --ragged-segments 0 --no-pcie --no-cpu-baseline > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 - $O/$tag.log $tag <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "commit", round(d["ms_per_step"] * 1e3, 2), "lease", round(d["lease"]["ms_per_pass"] * 1e3, 2),
      "fused", round(d["lease"]["fused_with_commit"]["roofline"]["avg_launch_ms"] * 1e3, 2), d["lease"]["parity_ok"], {k: v for k, v in d.items() if "parity" in k})
PY
done
done
