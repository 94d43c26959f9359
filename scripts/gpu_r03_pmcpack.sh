# PMC passes (separate runs, kernel trace only) for crc_pack_kernel on ragged 64-2048 B frames, then
# the stitch timing probe (debug build, printf).
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03pk
mkdir -p $OUT && export TMPDIR=/tmp && cd /tmp
run() { local name=$1 ctrs=$2; shift 2
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$OUT/pmc/$name" -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/scripts/prof_kernels.py "$@" > "$OUT/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run pack_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what crcragged --segments 64 --iters 3
run pack_c "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA" --what crcragged --segments 64 --iters 3
run pack_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what crcragged --segments 64 --iters 3
cd $GRAFT_REPO_ROOT
RATIS_HIP_LIB=$PWD/ratis_amd/lib/ab/libratis_hip_stats.so timeout -k 10 120 python scripts/prof_kernels.py --what ragged_read --segments 16 --iters 2 > $OUT/stitch_probe.txt 2>&1
echo probe rc=$?
grep seg $OUT/stitch_probe.txt | head -12
