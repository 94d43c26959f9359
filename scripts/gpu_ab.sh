# A/B of library builds on one box: RATIS_HIP_LIB=<build> microbench, alternating, 2 rounds
mkdir -p gpurun_out/ab && export TMPDIR=/tmp
SECTIONS=${SECTIONS:-crc,crcshape,ragread}
for r in 1 2; do
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/*.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/microbench.py --only $SECTIONS --segments ${SEGS:-64} --rounds 3 > gpurun_out/ab/${tag}_$r.log 2>&1 || { tail -20 gpurun_out/ab/${tag}_$r.log; exit 1; }
  echo "== $tag round $r"; grep -v calibration gpurun_out/ab/${tag}_$r.log | grep kernel | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['kernel'], d.get('shape', ''), d['median_GBps'])"
done
done
