# Round 4: the bitop3 CRC folds without the packed kernel's two register sets (x3only) against
# the shipped build and x3 (both), then two PMC passes (separate runs, kernel trace only) of the
# frame-API packed kernel on the x3only build: issue / wait / LDS counters.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04x3b}
mkdir -p $O && export TMPDIR=/tmp
AB=$R/ratis_amd/lib/ab/libratis_hip_x3only.so
RATIS_HIP_LIB=$AB timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py > $O/pytest_ab.log 2>&1 || { tail -60 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
n=0
for lib in $R/ratis_amd/lib/libratis_hip.so $AB $R/ratis_amd/lib/ab/libratis_hip_x3.so $R/ratis_amd/lib/libratis_hip.so $AB $R/ratis_amd/lib/ab/libratis_hip_x3.so; do
  n=$((n + 1)); tag=$(basename $lib .so)_$n
  for w in "ragged_read --segments 128" "crcragged --segments 64"; do
    wt=$(echo $w | cut -d' ' -f1)
    cd /tmp && RATIS_HIP_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/${wt}_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what $w --iters 6 > $O/${wt}_$tag.log 2>&1 || { tail -5 $O/${wt}_$tag.log; exit 1; }
  done
done
cd /tmp
RATIS_HIP_LIB=$AB timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d $O/pmc_a -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what crcragged --segments 64 --iters 4 > $O/pmc_a.log 2>&1 || { tail -5 $O/pmc_a.log; exit 1; }
RATIS_HIP_LIB=$AB timeout -s KILL 90 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE -d $O/pmc_b -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what crcragged --segments 64 --iters 4 > $O/pmc_b.log 2>&1 || { tail -5 $O/pmc_b.log; exit 1; }
echo done
