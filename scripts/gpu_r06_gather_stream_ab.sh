# Round 6 A/B: the REGION record gather on the table stream (default) against the side stream behind
# an event (side: RH_GATHER_SIDE=1) -- the table legs' host wait (commit and watch, AUTO sink) and the
# 1M-delta streaming leg, two alternating rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06gsab}
mkdir -p $O
for round in 1 2; do
  for lib in default side; do
    if [ $lib = default ]; then L=$R/ratis_amd/lib/libratis_hip.so; else L=$R/ratis_amd/lib/ab/libratis_hip_$lib.so; fi
    RATIS_HIP_LIB=$L timeout -k 10 200 python3 -u $R/scripts/table_bench.py --reps 8 --fracs 1.0,0.25,0.1 > $O/table_${lib}_$round.log 2>&1 || exit 1
    RATIS_HIP_LIB=$L timeout -k 10 200 python3 -u $R/scripts/stream_bench.py > $O/stream_${lib}_$round.log 2>&1 || exit 1
    echo "$lib $round done"
  done
done
