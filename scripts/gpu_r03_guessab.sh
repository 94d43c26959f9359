# Framing change: framing / read parity, then the read-launch + framing A/B against the previous build
# and the kernel split
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03g && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py tests/test_gpu_segment.py tests/test_gpu_crc.py > $R/gpurun_out/r03g/pytest.log 2>&1 || { tail -20 $R/gpurun_out/r03g/pytest.log; exit 1; }
tail -1 $R/gpurun_out/r03g/pytest.log
rm -rf gpurun_out/ab
SEGS=128 SECTIONS=ragread,framing bash scripts/gpu_ab.sh > gpurun_out/r03g/ab.txt 2>&1 || { tail -30 gpurun_out/r03g/ab.txt; exit 1; }
python3 scripts/ab_table.py
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r03g/prof -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 6 > $R/gpurun_out/r03g/prof.log 2>&1 || { tail -20 $R/gpurun_out/r03g/prof.log; exit 1; }
cd $R && python3 scripts/prof_summary.py gpurun_out/r03g/prof/run_kernel_trace.csv --top 10
