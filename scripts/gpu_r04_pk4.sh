# Round 4: packed CRC kernel over four fold chains of 4 words (tree join) against the shipped two
# chains of 8: CRC / read-path GPU tests on the A/B build, then kernel traces of the ragged read
# launch and the frame-API packed kernel, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04pk4}
mkdir -p $O && export TMPDIR=/tmp
AB=$R/ratis_amd/lib/ab/libratis_hip_${2:-pk4}.so
RATIS_HIP_LIB=$AB timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py > $O/pytest_ab.log 2>&1 || { tail -60 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
n=0
for lib in $R/ratis_amd/lib/libratis_hip.so $AB $R/ratis_amd/lib/libratis_hip.so $AB $R/ratis_amd/lib/libratis_hip.so $AB; do
  n=$((n + 1)); tag=$(basename $lib .so)_$n
  for w in "ragged_read --segments 128" "crcragged --segments 64"; do
    wt=$(echo $w | cut -d' ' -f1)
    cd /tmp && RATIS_HIP_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/${wt}_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what $w --iters 6 > $O/${wt}_$tag.log 2>&1 || { tail -5 $O/${wt}_$tag.log; exit 1; }
  done
  cd $R
done
python3 scripts/ab_parse.py $O crc_pack
