# Round 6 A/B: delta batches of up to 65536 applied from the pinned slot in place (zc64k:
# RH_DELTA_ZC_MAX=65536) against 4096 (default; larger batches by DMA into HBM first) -- the table
# legs' host wait from _async to the records at 3 / 1 / 0.3 % dirty, two alternating rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06zcab}
mkdir -p $O
for round in 1 2; do
  for lib in ${LIBS:-default zc64k}; do
    if [ $lib = default ]; then L=$R/ratis_amd/lib/libratis_hip.so; else L=$R/ratis_amd/lib/ab/libratis_hip_$lib.so; fi
    RATIS_HIP_LIB=$L timeout -k 10 200 python3 -u $R/scripts/table_bench.py --reps 8 --fracs ${FRACS:-0.03,0.01,0.003} > $O/${lib}_$round.log 2>&1 || exit 1
    echo "$lib $round done"
  done
done
