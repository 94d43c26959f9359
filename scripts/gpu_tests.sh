# full GPU test suite (one process)
mkdir -p gpurun_out/r02t && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/r02t/pytest.log 2>&1 || { tail -40 gpurun_out/r02t/pytest.log; exit 1; }
tail -1 gpurun_out/r02t/pytest.log
