# Parallel merge precompute + slot-mode packed CRC: framing / read-path parity, then the read-launch
# kernel split (rocprof) and the A/B microbench against the round-start split build
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03s && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_crc.py tests/test_gpu_segread.py tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py > $R/gpurun_out/r03s/pytest.log 2>&1 || { tail -30 $R/gpurun_out/r03s/pytest.log; exit 1; }
tail -1 $R/gpurun_out/r03s/pytest.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03s/prof -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 6 > $R/gpurun_out/r03s/prof.log 2>&1 || { tail -20 $R/gpurun_out/r03s/prof.log; exit 1; }
cd $R
python3 scripts/prof_summary.py gpurun_out/r03s/prof/run_kernel_trace.csv --top 16
rm -rf gpurun_out/ab
SEGS=128 SECTIONS=crcshape,ragread bash scripts/gpu_ab.sh > gpurun_out/r03s/ab.txt 2>&1 || { tail -30 gpurun_out/r03s/ab.txt; exit 1; }
python3 scripts/ab_table.py
