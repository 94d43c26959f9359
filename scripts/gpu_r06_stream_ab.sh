# Round 6 A/B: the delta streaming leg (1M deltas per step, pipelined) with every batch applied from
# the pinned slot in place (zc1m: RH_DELTA_ZC_MAX=1048576) against the DMA of large batches (default).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06streamab}
mkdir -p $O
for round in 1 2; do
  for lib in ${LIBS:-default zc1m}; do
    if [ $lib = default ]; then L=$R/ratis_amd/lib/libratis_hip.so; else L=$R/ratis_amd/lib/ab/libratis_hip_$lib.so; fi
    RATIS_HIP_LIB=$L timeout -k 10 200 python3 -u $R/scripts/stream_bench.py > $O/${lib}_$round.log 2>&1 || exit 1
    echo "$lib $round done"
  done
done
