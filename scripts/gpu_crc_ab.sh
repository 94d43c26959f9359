# CRC change: parity first, then the A/B microbench (product build vs window-only build)
mkdir -p gpurun_out/r02f && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py > gpurun_out/r02f/pytest.log 2>&1 || { tail -40 gpurun_out/r02f/pytest.log; exit 1; }
tail -1 gpurun_out/r02f/pytest.log
bash scripts/gpu_ab.sh
