# Round 3: refill guess kernel -- framing / read-path parity, then A/B of the guess variants.
set -o pipefail
mkdir -p gpurun_out/r03g && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py tests/test_gpu_segment.py > gpurun_out/r03g/pytest.log 2>&1 || { tail -40 gpurun_out/r03g/pytest.log; exit 1; }
tail -3 gpurun_out/r03g/pytest.log
for r in 1 2; do
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/*.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/microbench.py --only framing,ragread --segments 128 --rounds 3 > gpurun_out/r03g/${tag}_$r.log 2>&1 || { tail -20 gpurun_out/r03g/${tag}_$r.log; exit 1; }
  echo "== $tag round $r"; grep -v calibration gpurun_out/r03g/${tag}_$r.log | grep kernel | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['kernel'], d.get('shape', ''), d['median_GBps'])"
done
done
