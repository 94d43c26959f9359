# read-path change: CRC / segread parity tests, then the A/B microbench (read launches)
mkdir -p gpurun_out/r02r && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py > gpurun_out/r02r/pytest.log 2>&1 || { tail -40 gpurun_out/r02r/pytest.log; exit 1; }
tail -1 gpurun_out/r02r/pytest.log
SECTIONS=ragread,readc5 bash scripts/gpu_ab.sh
