# Round 5: a subset (or all) of the GPU test suite, one pytest process, every test under a timeout.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05t}
shift
mkdir -p $O && export TMPDIR=/tmp
cd $R
timeout -k 10 ${TO:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${@:-tests} > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
