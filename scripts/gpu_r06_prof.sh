# Round 6 (the round-5 recipe at HEAD): per-dispatch kernel trace of the bench run with every timed leg marked (roctx ranges,
# scripts/prof_legs.py), and the headline kernel's size sweep under the same trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06prof}
mkdir -p $O && export TMPDIR=/tmp
cd /tmp
if [ "${SWEEP:-1}" = 1 ]; then
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace -d $O/sweep_prof -o run --output-format csv -- python3 -u $R/scripts/commit_sweep.py ${SWEEP_ARGS:-} > $O/sweep.log 2>&1 || { tail -30 $O/sweep.log; exit 1; }
cat $O/sweep.log | grep -v "^W" | tail -12
python3 $R/scripts/prof_legs.py $O/sweep_prof > $O/sweep_legs.md || exit 1
fi
if [ "${BENCH:-1}" = 1 ]; then
# the same bench unprofiled first: the table legs' ms_evaluation comes from HIP events stamped by
# hipExtLaunchKernel, which the profiler's own completion signals stretch by ~4 us per launch; the
# legs table compares the trace with this run's line
timeout -k 10 600 python3 -u $R/bench.py ${BENCH_ARGS:-} > $O/bench_plain.log 2>&1 || { tail -30 $O/bench_plain.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --marker-trace --stats -d $O/bench_prof -o run --output-format csv -- python3 -u $R/bench.py ${BENCH_ARGS:-} > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
python3 $R/scripts/prof_legs.py $O/bench_prof $O/bench_plain.log > $O/bench_legs.md || exit 1
tail -20 $O/bench_legs.md
fi
