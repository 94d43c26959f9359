# Stitch merge-walk window A/B: 8 KiB (HEAD) vs 16 and 32 KiB windows (RH_MERGE_WIN): parity on each build, then read launch + framing A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03mw && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py tests/test_gpu_segment.py tests/test_gpu_crc.py > $R/gpurun_out/r03mw/pytest_head.log 2>&1 || { tail -20 $R/gpurun_out/r03mw/pytest_head.log; exit 1; }
tail -1 $R/gpurun_out/r03mw/pytest_head.log
for b in w16 w32; do
  RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_$b.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py tests/test_gpu_segment.py > $R/gpurun_out/r03mw/pytest_$b.log 2>&1 || { tail -20 $R/gpurun_out/r03mw/pytest_$b.log; exit 1; }
  tail -1 $R/gpurun_out/r03mw/pytest_$b.log
done
rm -rf gpurun_out/ab
SEGS=${SEGS:-256} SECTIONS=ragread,framing bash scripts/gpu_ab.sh > gpurun_out/r03mw/ab.txt 2>&1 || { tail -30 gpurun_out/r03mw/ab.txt; exit 1; }
python3 scripts/ab_table.py

