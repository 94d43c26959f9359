# PMC passes (separate runs, kernel trace only) over the ragged read launch, for the guess kernel
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03pg
mkdir -p $OUT && export TMPDIR=/tmp && cd /tmp
run() { local name=$1 ctrs=$2; shift 2
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmc/$name" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_kernels.py "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run g_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" --what ragged_read --segments 64 --iters 2
run g_b "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_INSTS_BRANCH" --what ragged_read --segments 64 --iters 2
