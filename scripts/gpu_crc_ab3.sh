# CRC change: CRC / read-path / framing parity, then A/B (config 5, frame shapes, read launches)
mkdir -p gpurun_out/r02f && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py tests/test_gpu_segment.py tests/test_gpu_framing_pieces.py > gpurun_out/r02f/pytest.log 2>&1 || { tail -40 gpurun_out/r02f/pytest.log; exit 1; }
tail -1 gpurun_out/r02f/pytest.log
SEGS=${SEGS:-128} SECTIONS=crc,crcshape,readc5,ragread bash scripts/gpu_ab.sh
