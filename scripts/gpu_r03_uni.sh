# Wave-uniform merge walk: parity (framing / read / CRC GPU tests) at the working tree, the stitch
# kernel under rocprofv3 on fallback-bearing data (walk_probe.py 256) for old (HEAD) and new, then
# the ragged read / framing A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03u && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_framing_pieces.py tests/test_gpu_segread.py tests/test_gpu_segment.py tests/test_gpu_crc.py > $R/gpurun_out/r03u/pytest_head.log 2>&1 || { tail -20 $R/gpurun_out/r03u/pytest_head.log; exit 1; }
tail -1 $R/gpurun_out/r03u/pytest_head.log
for b in new old; do
  lib=$R/ratis_amd/lib/ab/libratis_hip_$b.so; [ $b = new ] && lib=$R/ratis_amd/lib/libratis_hip.so
  (cd /tmp && RATIS_HIP_LIB=$lib timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/r03u/$b -o run --output-format csv -- python3 $R/scripts/walk_probe.py 256) > $R/gpurun_out/r03u/$b.log 2>&1 || { tail -20 $R/gpurun_out/r03u/$b.log; exit 1; }
done
rm -rf gpurun_out/ab
SEGS=${SEGS:-256} SECTIONS=ragread,framing bash scripts/gpu_ab.sh > gpurun_out/r03u/ab.txt 2>&1 || { tail -30 gpurun_out/r03u/ab.txt; exit 1; }
python3 scripts/ab_table.py
