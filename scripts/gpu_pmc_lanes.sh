# PMC passes over the CRC lane kernels (uniform 516 B frames, ragged 64-2048 B) and the window
# kernel (uniform 4096 B) -- one counter set per rocprofv3 run
set -u
OUT=gpurun_out/pmc_lanes; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name counters args...
  local name=$1 ctrs=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d $OUT/$name -o run --output-format csv -- python3 scripts/prof_kernels.py "$@" > $OUT/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; exit 1; fi
}
for shape in "s516 --what crcshape --frame-size 516" "rag --what crcragged" "s4096 --what crcshape --frame-size 4096"; do
  set -- $shape; tag=$1; shift
  run ${tag}_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS" "$@" --segments 32 --iters 3
  run ${tag}_b "FETCH_SIZE GRBM_GUI_ACTIVE" "$@" --segments 32 --iters 3
  run ${tag}_c "SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU" "$@" --segments 32 --iters 3
done
echo PMCDONE
