# guess-pass refill variant: its framing / read-path parity, then same-box A/B against the product
mkdir -p gpurun_out/r02r && export TMPDIR=/tmp
RATIS_HIP_LIB=$PWD/ratis_amd/lib/ab/libratis_hip_refill.so timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py tests/test_gpu_segread.py > gpurun_out/r02r/pytest.log 2>&1 || { tail -40 gpurun_out/r02r/pytest.log; exit 1; }
tail -1 gpurun_out/r02r/pytest.log
SEGS=${SEGS:-128} SECTIONS=framing,ragread bash scripts/gpu_ab.sh > /dev/null
python scripts/ab_table.py
