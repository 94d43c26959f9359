# Round 6 A/B of the tick (RATIS_HIP_LIB: default vs ratis_amd/lib/ab/libratis_hip_rec.so, the build under test), e.g. the result-set event completed by the launch itself vs recorded
# after it (rec: RH_TICK_STOP_EVENT=0); tick_breakdown.py twice each, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06tickab}
mkdir -p $O
for round in 1 2; do
  for lib in default rec; do
    if [ $lib = default ]; then L=$R/ratis_amd/lib/libratis_hip.so; else L=$R/ratis_amd/lib/ab/libratis_hip_$lib.so; fi
    RATIS_HIP_LIB=$L timeout -k 10 200 python3 -u $R/scripts/tick_breakdown.py > $O/${lib}_$round.json 2> $O/${lib}_$round.err || exit 1
  done
done
