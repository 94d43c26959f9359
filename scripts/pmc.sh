#!/bin/bash
# PMC passes (separate rocprofv3 runs, kernel-trace only, no sys/runtime trace) for the two
# hot kernels.  Output under gpurun_out/$RUN_TAG/pmc/<name>/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/${RUN_TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocprofv3 -L > "$OUT/counters_list.txt" 2>&1 || true
run() {  # name "counters" driver-args...
  local name=$1 ctrs=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmc/$name" -o run --output-format csv -- python3 "$R/scripts/prof_kernels.py" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  if [ $rc -ge 124 ]; then exit $rc; fi
}
run crc_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" --what crc
run crc_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what crc
run crc_c "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM" --what crc
run crc_w "WRITE_SIZE" --what crc
run commit_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what commit
run commit_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what commit
run commit_w "WRITE_SIZE" --what commit
if [ "${FRAMING:-1}" = "1" ]; then
  run framing_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD" --what framing --segments 64
  run framing_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what framing --segments 64
  run framing_w "WRITE_SIZE" --what framing --segments 64
fi
if [ "${LEASE:-1}" = "1" ]; then
  run lease_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what lease --iters 8
  run lease_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what lease --iters 8
  run lease_w "WRITE_SIZE" --what lease --iters 8
fi
echo PMCDONE
