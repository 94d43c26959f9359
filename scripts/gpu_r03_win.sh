# Guess survival window A/B (4 / 3 / 2 gmax): parity of the framing tests on each build, then the
# read-launch microbench, then the kernel split of the 2-gmax build
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03w && export TMPDIR=/tmp
for b in ab/libratis_hip_win2 ab/libratis_hip_win3; do
  RATIS_HIP_LIB=$R/ratis_amd/lib/$b.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py > $R/gpurun_out/r03w/pytest_$(basename $b).log 2>&1 || { tail -20 $R/gpurun_out/r03w/pytest_$(basename $b).log; exit 1; }
  tail -1 $R/gpurun_out/r03w/pytest_$(basename $b).log
done
rm -rf gpurun_out/ab
SEGS=128 SECTIONS=ragread bash scripts/gpu_ab.sh > gpurun_out/r03w/ab.txt 2>&1 || { tail -30 gpurun_out/r03w/ab.txt; exit 1; }
python3 scripts/ab_table.py
cd /tmp
RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_win2.so timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r03w/prof -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 6 > $R/gpurun_out/r03w/prof.log 2>&1 || { tail -20 $R/gpurun_out/r03w/prof.log; exit 1; }
cd $R && python3 scripts/prof_summary.py gpurun_out/r03w/prof/run_kernel_trace.csv --top 12
