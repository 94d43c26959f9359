# Round 4: the new GPU tests (JNI harness, pump fallback, list mode, stamp) then the whole suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04l}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_jni.py tests/test_gpu_pump.py tests/test_gpu_segread.py::test_fused_ragged_bench_scale_against_oracle > $O/pytest_new.log 2>&1 || { tail -60 $O/pytest_new.log; exit 1; }
tail -1 $O/pytest_new.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
