# Round 4 final check at HEAD: full GPU suite, smoke, the bench line, then PMC passes (separate
# kernel-trace-only runs) of the headline commit kernel, the frame CRC kernel and the lease kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04z}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python -u bench.py > $O/bench.log 2>&1 || { tail -30 $O/bench.log; exit 1; }
echo bench done
RUN_TAG=${1:-r04z} FRAMING=0 bash $R/scripts/pmc.sh > $O/pmc_passes.log 2>&1 || { tail -20 $O/pmc_passes.log; exit 1; }
tail -12 $O/pmc_passes.log
