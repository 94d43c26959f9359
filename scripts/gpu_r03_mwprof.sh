# Stitch kernel time with the merge-walk window at 8 (HEAD) / 16 / 32 KiB on data whose segments
# include false-survivor fallbacks (walk_probe.py, seed 5): rocprofv3 kernel trace per build
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03mp && cd /tmp && export TMPDIR=/tmp
for b in head w16 w32; do
  lib=$R/ratis_amd/lib/ab/libratis_hip_$b.so; [ $b = head ] && lib=$R/ratis_amd/lib/libratis_hip.so
  RATIS_HIP_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03mp/$b -o run --output-format csv -- python3 $R/scripts/walk_probe.py 256 > $R/gpurun_out/r03mp/$b.log 2>&1 || { tail -20 $R/gpurun_out/r03mp/$b.log; exit 1; }
  tail -1 $R/gpurun_out/r03mp/$b.log
done
