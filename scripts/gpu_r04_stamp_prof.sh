# Round 4: where the fixed cost of rh_crc32c_stamp_host goes (kernel + copy trace), and the table
# list-mode kernel after the prefix fix.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04g
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_write_stamp.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/sprof -o run --output-format csv -- python3 $R/scripts/stamp_bench.py > $O/sprof.log 2>&1 || { tail -20 $O/sprof.log; exit 1; }
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/tprof -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 4 > $O/tprof.log 2>&1 || { tail -20 $O/tprof.log; exit 1; }
tail -1 $O/sprof.log | cut -c1-400
echo done
