# Round 3 evidence: rocprofv3 kernel trace + stats of the bench, and PMC passes (separate runs,
# kernel-trace only) for the resident-table kernel and the lease kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03p && export TMPDIR=/tmp && cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03p/bench_prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/r03p/bench.log 2>&1 || { tail -20 $R/gpurun_out/r03p/bench.log; exit 1; }
echo bench-prof done
cd $R
RUN_TAG=r03p FRAMING=0 LEASE=0 bash -c '
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03p
run() { local name=$1 ctrs=$2; shift 2
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmc/$name" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_kernels.py "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run table_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what table --iters 6
run table_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what table --iters 6
run table_w "WRITE_SIZE" --what table --iters 6
run lease_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what lease --iters 8
run lease_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what lease --iters 8
run lease_w "WRITE_SIZE" --what lease --iters 8
run ragged_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU" --what ragged_read --segments 64 --iters 2
run ragged_b "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD" --what ragged_read --segments 64 --iters 2
'
echo PMCDONE
