# Round 4: bench-scale ragged read launch (256 x 32 MiB), shipped build vs the build before the
# bitop3 CRC change (prebit), alternating on one box, HIP events around 10 launches x 3 rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04rrab}
mkdir -p $O
for lib in libratis_hip.so ab/libratis_hip_prebit.so libratis_hip.so ab/libratis_hip_prebit.so libratis_hip.so ab/libratis_hip_prebit.so; do
  RATIS_HIP_LIB=$R/ratis_amd/lib/$lib timeout -k 10 150 python -u scripts/rr_time.py >> $O/rr.log 2>&1 || { tail -20 $O/rr.log; exit 1; }
  tail -1 $O/rr.log
done
