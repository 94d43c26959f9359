# Round 4: packed CRC kernel prefetch depth -- x3pp (bitop3 folds, two register sets, 16 waves/CU)
# and d2 (three register sets, 12 waves/CU) against the shipped build: CRC / read-path GPU tests on
# both A/B builds, then kernel traces of the ragged read launch and the frame-API packed kernel,
# alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04dp}
mkdir -p $O && export TMPDIR=/tmp
for v in x3pp d2; do
  RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py > $O/pytest_$v.log 2>&1 || { tail -60 $O/pytest_$v.log; exit 1; }
  tail -1 $O/pytest_$v.log
done
n=0
for lib in $R/ratis_amd/lib/libratis_hip.so $R/ratis_amd/lib/ab/libratis_hip_x3pp.so $R/ratis_amd/lib/ab/libratis_hip_d2.so $R/ratis_amd/lib/libratis_hip.so $R/ratis_amd/lib/ab/libratis_hip_x3pp.so $R/ratis_amd/lib/ab/libratis_hip_d2.so; do
  n=$((n + 1)); tag=$(basename $lib .so)_$n
  for w in "ragged_read --segments 128" "crcragged --segments 64"; do
    wt=$(echo $w | cut -d' ' -f1)
    cd /tmp && RATIS_HIP_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/${wt}_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what $w --iters 6 > $O/${wt}_$tag.log 2>&1 || { tail -5 $O/${wt}_$tag.log; exit 1; }
  done
  cd $R
done
echo done
