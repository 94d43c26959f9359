# Kernel-boundary probe: an empty kernel between piece_walk and piece_stitch (A/B build)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03pr && export TMPDIR=/tmp && cd /tmp
RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_probe.so timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/r03pr/prof -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 3 > $R/gpurun_out/r03pr/prof.log 2>&1 || { tail -20 $R/gpurun_out/r03pr/prof.log; exit 1; }
cd $R && python3 scripts/prof_summary.py gpurun_out/r03pr/prof/run_kernel_trace.csv --top 14
