# PMC passes (separate runs, kernel trace only) over the ragged read launch: its HBM traffic
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03x/pmc && export TMPDIR=/tmp && cd /tmp
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/r03x/pmc/rr_b -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 64 --iters 4 > $R/gpurun_out/r03x/pmc/rr_b.log 2>&1 || { tail -5 $R/gpurun_out/r03x/pmc/rr_b.log; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/r03x/pmc/rr_w -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 64 --iters 4 > $R/gpurun_out/r03x/pmc/rr_w.log 2>&1 || { tail -5 $R/gpurun_out/r03x/pmc/rr_w.log; exit 1; }
echo PMCDONE
