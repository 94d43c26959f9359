# Packed CRC kernel change: CRC / read parity, A/B (CRC shapes, read launch) against the previous
# build, then one FETCH_SIZE pass over the ragged CRC (HBM bytes per launch)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r03t && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_crc.py tests/test_gpu_segread.py tests/test_gpu_framing_pieces.py > $R/gpurun_out/r03t/pytest.log 2>&1 || { tail -20 $R/gpurun_out/r03t/pytest.log; exit 1; }
tail -1 $R/gpurun_out/r03t/pytest.log
rm -rf gpurun_out/ab
SEGS=128 SECTIONS=crcshape,ragread bash scripts/gpu_ab.sh > gpurun_out/r03t/ab.txt 2>&1 || { tail -30 gpurun_out/r03t/ab.txt; exit 1; }
python3 scripts/ab_table.py
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $R/gpurun_out/r03t/pmc/pack_b -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what crcragged --segments 64 --iters 3 > $R/gpurun_out/r03t/pack_b.log 2>&1; echo pmc rc=$?
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $R/gpurun_out/r03t/pmc/pack_w -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what crcragged --segments 64 --iters 3 > $R/gpurun_out/r03t/pack_w.log 2>&1; echo pmc rc=$?
