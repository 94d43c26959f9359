# Round 5: pump-tick latency A/B (scripts/tick_bench.py per library, alternating, 2 rounds).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05k}
mkdir -p $O && export TMPDIR=/tmp
cd $R
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $(ls $R/ratis_amd/lib/ab/*.so 2>/dev/null); do
  tag=$(basename $lib .so)_$r
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/tick_bench.py > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo $tag $(grep '^{' $O/$tag.log | tail -1)
done
done
