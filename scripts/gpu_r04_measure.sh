# Round 4 evidence at HEAD: the default bench run, a rocprofv3 kernel trace + stats of the bench,
# and PMC passes (separate runs, kernel-trace only) for the resident-table evaluation and the
# ragged read launch.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r04p}
O=$R/gpurun_out/$T
mkdir -p $O/pmc && export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
echo bench done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/bench_prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $O/bench_prof.log 2>&1 || { tail -20 $O/bench_prof.log; exit 1; }
echo bench-prof done
run() { local name=$1 ctrs=$2; shift 2
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctrs -d "$O/pmc/$name" -o run --output-format csv -- python3 $R/scripts/prof_kernels.py "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then exit $rc; fi; }
run table_a "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD" --what table --iters 6
run table_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what table --iters 6
run table_w "WRITE_SIZE" --what table --iters 6
run rr_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what ragged_read --segments 64 --iters 4
run rr_w "WRITE_SIZE" --what ragged_read --segments 64 --iters 4
echo PMCDONE
