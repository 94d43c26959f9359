# Round 5: PMC passes (one rocprofv3 run per counter group, kernel-trace only) of the kernels whose
# rooflines carry `traffic`: the resident-table evaluation (100 % dirty), the headline commit
# kernel, the lease kernel; summarised by scripts/pmc_summary.py.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05pmc}
mkdir -p $O/pmc && export TMPDIR=/tmp
cd /tmp
run() { local name=$1 ctrs=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$O/pmc/$name" -o run --output-format csv -- python3 $R/scripts/prof_kernels.py "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -20 "$O/$name.log"; exit $rc; fi; }
run table_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what table --iters 6
run table_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what table --iters 6
run table_w "WRITE_SIZE" --what table --iters 6
run commit_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what commit --iters 8
run commit_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what commit --iters 8
run commit_w "WRITE_SIZE" --what commit --iters 8
run lease_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what lease --iters 8
run lease_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what lease --iters 8
run lease_w "WRITE_SIZE" --what lease --iters 8
grep -h "alg_bytes" $O/table_b.log | tail -1
python3 $R/scripts/pmc_summary.py $O/pmc --out $O/pmc_traffic.json && echo PMCDONE
