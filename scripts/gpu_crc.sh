# CRC kernel change: parity tests, microbench (config 5 + frame-shape sweep), bench CRC legs
mkdir -p gpurun_out/r02f && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py tests/test_gpu_framing_pieces.py tests/test_gpu_segment.py > gpurun_out/r02f/pytest.log 2>&1 || { tail -40 gpurun_out/r02f/pytest.log; exit 1; }
tail -1 gpurun_out/r02f/pytest.log
timeout -k 10 300 python -u scripts/microbench.py --only crc,crcshape --segments 64 --rounds 3 > gpurun_out/r02f/micro.log 2>&1 || { tail -30 gpurun_out/r02f/micro.log; exit 1; }
grep crc32c gpurun_out/r02f/micro.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('shape', 'config5'), d['median_GBps'])"
timeout -k 10 400 python -u bench.py --steps 10 --no-lease --no-pcie --no-cpu-baseline > gpurun_out/r02f/bench.log 2>&1 || { tail -20 gpurun_out/r02f/bench.log; exit 1; }
tail -1 gpurun_out/r02f/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['crc32c']; print('crc', c['GBps'], c['roofline']['frac'], c['parity_ok'], 'read', c['read_path']['read_launch_GBps'], 'ragged', json.dumps(c['read_path'].get('ragged'))[:700])"
