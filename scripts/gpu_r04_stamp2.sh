# Round 4: serial stamp kernel with the next 128-byte round prefetched -- stamp / CRC tests, the
# stamp bench, and a kernel + copy trace of it.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04x}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_write_stamp.py tests/test_gpu_crc.py tests/test_gpu_jni.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 200 python -u scripts/stamp_bench.py > $O/stamp.log 2>&1 || { tail -20 $O/stamp.log; exit 1; }
tail -1 $O/stamp.log | cut -c1-700
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/sprof -o run --output-format csv -- python3 $R/scripts/stamp_bench.py > $O/sprof.log 2>&1 || { tail -20 $O/sprof.log; exit 1; }
echo done
