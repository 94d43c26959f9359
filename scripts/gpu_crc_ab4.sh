# CRC prepass change: CRC / read-path parity, then A/B (CRC shapes, read launches)
mkdir -p gpurun_out/r02f && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py > gpurun_out/r02f/pytest.log 2>&1 || { tail -40 gpurun_out/r02f/pytest.log; exit 1; }
tail -1 gpurun_out/r02f/pytest.log
SEGS=${SEGS:-128} SECTIONS=crcshape,ragread bash scripts/gpu_ab.sh > /dev/null
python scripts/ab_table.py
