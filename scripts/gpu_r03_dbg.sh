# kernel split of the ragged read launch at HEAD (rocprof kernel trace)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03d && export TMPDIR=/tmp && cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r03d/prof -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 3 > $R/gpurun_out/r03d/prof.log 2>&1 || { tail -20 $R/gpurun_out/r03d/prof.log; exit 1; }
cd $R && python3 scripts/prof_summary.py gpurun_out/r03d/prof/run_kernel_trace.csv --top 14
