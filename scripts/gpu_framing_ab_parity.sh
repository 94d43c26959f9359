# framing A/B: every ratis_amd/lib/ab build's framing / read-path parity, then the same-box A/B
mkdir -p gpurun_out/r02f && export TMPDIR=/tmp
for lib in ratis_amd/lib/ab/*.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$PWD/$lib timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py tests/test_gpu_segread.py > gpurun_out/r02f/pytest_$tag.log 2>&1 || { tail -40 gpurun_out/r02f/pytest_$tag.log; exit 1; }
  echo "$tag: $(tail -1 gpurun_out/r02f/pytest_$tag.log)"
done
SEGS=${SEGS:-128} SECTIONS=${SECTIONS:-framing,ragread} bash scripts/gpu_ab.sh > /dev/null
python scripts/ab_table.py
