# Framing parity + microbench + rocprof, and the H2D probe (delta streaming bound).
mkdir -p gpurun_out/r02d && export TMPDIR=/tmp
timeout -k 10 60 ./scripts/h2d_probe > gpurun_out/r02d/h2d_probe.log 2>&1 || { cat gpurun_out/r02d/h2d_probe.log; exit 1; }
cat gpurun_out/r02d/h2d_probe.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py tests/test_gpu_segread.py > gpurun_out/r02d/pytest.log 2>&1 || { tail -40 gpurun_out/r02d/pytest.log; exit 1; }
tail -3 gpurun_out/r02d/pytest.log
timeout -k 10 300 python -u scripts/microbench.py --only framing --segments 256 --rounds 3 > gpurun_out/r02d/micro.log 2>&1 || exit 1
cat gpurun_out/r02d/micro.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r02d/prof -o run --output-format csv -- python3 scripts/microbench.py --only framing --segments 256 --rounds 1 --iters 3 > gpurun_out/r02d/prof.log 2>&1
