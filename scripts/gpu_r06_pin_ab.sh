# Round 6 A/B: AUTO's list evaluations writing their records into the pinned lists directly at any
# size (pinall) vs from 8192 marked rows in REGION mode + the gather (default): what the host waits
# for (async -> records in the pinned lists), two alternating rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06pinab}
mkdir -p $O
for round in 1 2; do
  for lib in default pinall; do
    if [ $lib = default ]; then L=$R/ratis_amd/lib/libratis_hip.so; else L=$R/ratis_amd/lib/ab/libratis_hip_$lib.so; fi
    RATIS_HIP_LIB=$L timeout -k 10 200 python3 -u $R/scripts/table_bench.py --reps 8 --fracs 0.1,0.03,0.01,0.003 > $O/${lib}_$round.log 2>&1 || exit 1
    echo "$lib $round done"
  done
done
