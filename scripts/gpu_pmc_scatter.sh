# PMC passes over the CRC prepass kernels in the ragged read launch (64 segments)
set -u
OUT=gpurun_out/pmc_scatter; mkdir -p $OUT; export TMPDIR=/tmp
run() {
  local name=$1 ctrs=$2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/$name -o run --output-format csv -- python3 scripts/prof_kernels.py --what ragged_read --segments 64 --iters 2 > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit 1; fi
}
run a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
run b "FETCH_SIZE GRBM_GUI_ACTIVE"
run w "WRITE_SIZE"
run c "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU"
python scripts/pmc_table.py $OUT/ crc_
