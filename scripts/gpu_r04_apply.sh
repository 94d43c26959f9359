# Round 4: summary byte set only while clear (delta apply) -- table tests, then the table leg
# under a kernel trace for the shipped build and the always-store A/B build.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04w}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_table_lease.py tests/test_gpu_pump.py > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_sumstore.so; do
  tag=$(basename $lib .so)
  cd /tmp && RATIS_HIP_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_$tag -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 4 --fracs 1.0,0.1,0.01 > $O/tb_$tag.log 2>&1 || { tail -30 $O/tb_$tag.log; exit 1; }
  cd $R
done
RATIS_HIP_LIB=$R/ratis_amd/lib/libratis_hip.so timeout -k 10 300 python -u bench.py --crc-segments 0 --no-lease --no-cpu-baseline --steps 10 > $O/bench_pcie.log 2>&1 || { tail -30 $O/bench_pcie.log; exit 1; }
echo done
