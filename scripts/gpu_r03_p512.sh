# 512 KiB piece tier A/B (mean frame >= 1 KiB) vs HEAD adaptive 128/256 KiB: parity on both builds (incl. the bench-scale ragged read test), then read launch + framing A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03p5 && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py tests/test_gpu_segment.py tests/test_gpu_crc.py > $R/gpurun_out/r03p5/pytest_head.log 2>&1 || { tail -20 $R/gpurun_out/r03p5/pytest_head.log; exit 1; }
tail -1 $R/gpurun_out/r03p5/pytest_head.log
for b in p512; do
  RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_$b.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py tests/test_gpu_segment.py > $R/gpurun_out/r03p5/pytest_$b.log 2>&1 || { tail -20 $R/gpurun_out/r03p5/pytest_$b.log; exit 1; }
  tail -1 $R/gpurun_out/r03p5/pytest_$b.log
done
rm -rf gpurun_out/ab
SEGS=${SEGS:-256} SECTIONS=ragread,framing bash scripts/gpu_ab.sh > gpurun_out/r03p5/ab.txt 2>&1 || { tail -30 gpurun_out/r03p5/ab.txt; exit 1; }
python3 scripts/ab_table.py

