# Round 3 close at HEAD: full GPU suite, smoke, bench, and the bench under rocprofv3 (kernel trace + stats)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03z && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $R/gpurun_out/r03z/pytest.log 2>&1 || { tail -40 $R/gpurun_out/r03z/pytest.log; exit 1; }
tail -1 $R/gpurun_out/r03z/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/gpurun_out/r03z/smoke.log 2>&1 || { tail -20 $R/gpurun_out/r03z/smoke.log; exit 1; }
tail -1 $R/gpurun_out/r03z/smoke.log
timeout -k 10 300 python -u bench.py > $R/gpurun_out/r03z/bench.log 2>&1 || { tail -30 $R/gpurun_out/r03z/bench.log; exit 1; }
echo bench done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03z/bench_prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/r03z/bench_prof.log 2>&1 || { tail -20 $R/gpurun_out/r03z/bench_prof.log; exit 1; }
echo bench-prof done
