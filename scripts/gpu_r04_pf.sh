# Round 4: packed CRC kernel loading the next task's frame-table entries during the current task
# (RH_PACK_PREFETCH=1, build pf) against the shipped build: CRC / read-path GPU tests on the A/B
# build, then the bench-scale ragged read launch (scripts/rr_time.py) and the frame-API packed
# kernel under a kernel trace, alternating on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04pf}
mkdir -p $O && export TMPDIR=/tmp
AB=$R/ratis_amd/lib/ab/libratis_hip_${2:-pf}.so
RATIS_HIP_LIB=$AB timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py tests/test_gpu_write_stamp.py > $O/pytest_ab.log 2>&1 || { tail -60 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
n=0
for lib in $R/ratis_amd/lib/libratis_hip.so $AB $R/ratis_amd/lib/libratis_hip.so $AB $R/ratis_amd/lib/libratis_hip.so $AB; do
  n=$((n + 1)); tag=$(basename $lib .so)_$n
  RATIS_HIP_LIB=$lib timeout -k 10 150 python -u scripts/rr_time.py >> $O/rr.log 2>&1 || { tail -20 $O/rr.log; exit 1; }
  tail -1 $O/rr.log
  cd /tmp && RATIS_HIP_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/crcragged_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what crcragged --segments 64 --iters 6 > $O/crcragged_$tag.log 2>&1 || { tail -5 $O/crcragged_$tag.log; exit 1; }
  cd $R
done
python3 scripts/ab_parse.py $O crc_pack
