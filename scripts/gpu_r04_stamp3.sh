# Round 4: rh_crc32c_stamp_host plans A/B (0 serial + copies, 1 window + copies, 2 window + mapped
# frame table / CRCs) -- stamp tests on the shipped build, the stamp bench per build, and a kernel +
# copy trace of the shipped build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04y}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_write_stamp.py tests/test_gpu_crc.py tests/test_gpu_jni.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in ratis_amd/lib/libratis_hip.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$R/$lib timeout -k 10 200 python -u scripts/stamp_bench.py > $O/stamp_$tag.log 2>&1 || { tail -20 $O/stamp_$tag.log; exit 1; }
  echo "== $tag"; tail -1 $O/stamp_$tag.log | cut -c1-420
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/sprof -o run --output-format csv -- python3 $R/scripts/stamp_bench.py > $O/sprof.log 2>&1 || { tail -20 $O/sprof.log; exit 1; }
echo done
