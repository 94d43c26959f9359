# tiled lease layout: lease parity tests, then the lease legs of bench.py in both layouts
mkdir -p gpurun_out/r02l && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_lease.py tests/test_gpu_table_lease.py tests/test_abi.py > gpurun_out/r02l/pytest.log 2>&1 || { tail -40 gpurun_out/r02l/pytest.log; exit 1; }
tail -1 gpurun_out/r02l/pytest.log
for lay in tiled plain tiled plain; do
timeout -k 10 400 python -u bench.py --steps 50 --crc-segments 0 --no-pcie --no-cpu-baseline --lease-layout $lay > gpurun_out/r02l/bench_$lay.log 2>&1 || { tail -20 gpurun_out/r02l/bench_$lay.log; exit 1; }
tail -1 gpurun_out/r02l/bench_$lay.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['lease']; print('$lay', 'commit', d['roofline']['frac'], 'lease', l['roofline']['frac'], l['ms_per_pass'], l['parity_ok'], 'fused', l['fused_with_commit']['roofline']['frac'], l['fused_with_commit']['parity_ok'])"
done
