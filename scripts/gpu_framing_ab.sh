# framing change: framing / read-path parity, then A/B (framing, ragged read launch)
mkdir -p gpurun_out/r02g && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py tests/test_gpu_segread.py > gpurun_out/r02g/pytest.log 2>&1 || { tail -40 gpurun_out/r02g/pytest.log; exit 1; }
tail -1 gpurun_out/r02g/pytest.log
SEGS=${SEGS:-128} SECTIONS=framing,ragread bash scripts/gpu_ab.sh > /dev/null
python scripts/ab_table.py
