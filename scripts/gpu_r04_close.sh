# Round 4 close at HEAD: full GPU suite and smoke (the in-tree library as shipped)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04c && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $R/gpurun_out/r04c/pytest.log 2>&1 || { tail -40 $R/gpurun_out/r04c/pytest.log; exit 1; }
tail -1 $R/gpurun_out/r04c/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $R/gpurun_out/r04c/smoke.log 2>&1 || { tail -20 $R/gpurun_out/r04c/smoke.log; exit 1; }
tail -1 $R/gpurun_out/r04c/smoke.log
timeout -k 10 300 python -u bench.py > $R/gpurun_out/r04c/bench.log 2>&1 || { tail -30 $R/gpurun_out/r04c/bench.log; exit 1; }
echo bench done
