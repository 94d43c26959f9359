# Round 3 at HEAD: full GPU suite, bench, then the ragged read launch's PMC passes (traffic)
set -o pipefail
mkdir -p gpurun_out/r03f && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03f/pytest.log 2>&1 || { tail -40 gpurun_out/r03f/pytest.log; exit 1; }
tail -1 gpurun_out/r03f/pytest.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03f/bench.log 2>&1 || { tail -30 gpurun_out/r03f/bench.log; exit 1; }
bash scripts/gpu_r03_pmcrr.sh
