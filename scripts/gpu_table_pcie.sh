# resident-table change: table parity tests, then the PCIe legs of bench.py (twice)
mkdir -p gpurun_out/r02tp && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table.py tests/test_gpu_table_lease.py > gpurun_out/r02tp/pytest.log 2>&1 || { tail -40 gpurun_out/r02tp/pytest.log; exit 1; }
tail -1 gpurun_out/r02tp/pytest.log
for i in 1 2; do
timeout -k 10 400 python -u bench.py --steps 20 --crc-segments 0 --no-lease --no-cpu-baseline > gpurun_out/r02tp/bench_$i.log 2>&1 || { tail -20 gpurun_out/r02tp/bench_$i.log; exit 1; }
tail -1 gpurun_out/r02tp/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); p=d['pcie']['delta_streaming']; print('delta', p['ms_per_step'], p['ms_per_step_runs'], p['stage_ms'], p['advanced_per_step'], 'full', d['pcie']['commit_ms_incl_pcie_full_snapshot'])"
done
