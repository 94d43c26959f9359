# Round 6 A/B: evaluation waves per gather workgroup (RH_GATHER_CHUNKS: 32 shipped, 8, 4) -- the
# REGION gather's time at 100 % and 10 % dirty (tile evaluations), two alternating rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06gab}
mkdir -p $O
for round in 1 2; do
  for lib in default g8 g4; do
    if [ $lib = default ]; then L=$R/ratis_amd/lib/libratis_hip.so; else L=$R/ratis_amd/lib/ab/libratis_hip_$lib.so; fi
    RATIS_HIP_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_${lib}_$round -o run --output-format csv -- python3 -u $R/scripts/table_bench.py --reps 8 --fracs 1.0,0.1 > $O/${lib}_$round.log 2>&1 || exit 1
    echo "$lib $round done"
  done
done
