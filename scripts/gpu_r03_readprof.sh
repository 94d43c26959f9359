# Kernel split of the ragged read launch (rocprofv3 kernel trace + stats), packed CRC plan
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03rp && export TMPDIR=/tmp && cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03rp/prof -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 6 > $R/gpurun_out/r03rp/prof.log 2>&1 || { tail -20 $R/gpurun_out/r03rp/prof.log; exit 1; }
python3 $R/scripts/prof_summary.py $R/gpurun_out/r03rp/prof/run_kernel_trace.csv --top 30
