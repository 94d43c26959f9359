# piece_walk_kernel duration at 4, 16, 64, 256 segments (concurrency probe), one rocprofv3 run each
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03w && cd /tmp && export TMPDIR=/tmp
for n in 4 16 64 256; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03w/n$n -o run -- python3 $R/scripts/walk_probe.py $n > $R/gpurun_out/r03w/n$n.log 2>&1 || { tail -20 $R/gpurun_out/r03w/n$n.log; exit 1; }
  tail -1 $R/gpurun_out/r03w/n$n.log
done
