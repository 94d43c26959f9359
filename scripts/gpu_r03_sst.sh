# Stitch tail probe: RH_STITCH_STATS build (per-segment pass / serial counts and 100 MHz times)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03s
for n in 64 256; do
  RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_sst.so timeout -k 10 180 python3 scripts/walk_probe.py $n > $R/gpurun_out/r03s/n$n.log 2>&1 || { tail -20 $R/gpurun_out/r03s/n$n.log; exit 1; }
  grep -c STITCH $R/gpurun_out/r03s/n$n.log
done
