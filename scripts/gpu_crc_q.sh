# lane-path width sweep: lanes per frame Q = 1..16 (RH_CRC_Q), parity at two widths, microbench each
mkdir -p gpurun_out/r02q && export TMPDIR=/tmp
for q in 4 16; do
RH_CRC_Q=$q timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py > gpurun_out/r02q/pytest_q$q.log 2>&1 || { tail -40 gpurun_out/r02q/pytest_q$q.log; exit 1; }
tail -1 gpurun_out/r02q/pytest_q$q.log
done
for q in 1 2 4 8 16; do
RH_CRC_Q=$q timeout -k 10 300 python -u scripts/microbench.py --only crc,crcshape --segments 64 --rounds 3 > gpurun_out/r02q/micro_q$q.log 2>&1 || { tail -30 gpurun_out/r02q/micro_q$q.log; exit 1; }
echo "== Q=$q"; grep crc32c gpurun_out/r02q/micro_q$q.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d.get('shape', 'config5'), d['median_GBps'])"
done
