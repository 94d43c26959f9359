# Tiled commit layout: parity tests, microbench (plain vs tiled), bench headline
mkdir -p gpurun_out/r02h && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_commit.py tests/test_gpu_lease.py > gpurun_out/r02h/pytest.log 2>&1 || { tail -40 gpurun_out/r02h/pytest.log; exit 1; }
tail -3 gpurun_out/r02h/pytest.log
timeout -k 10 300 python -u scripts/microbench.py --only commit --rounds 5 > gpurun_out/r02h/micro.log 2>&1 || { tail -20 gpurun_out/r02h/micro.log; exit 1; }
cat gpurun_out/r02h/micro.log
timeout -k 10 400 python -u bench.py --no-pcie --no-cpu-baseline --crc-segments 0 --ragged-segments 0 > gpurun_out/r02h/bench.log 2>&1 || { tail -20 gpurun_out/r02h/bench.log; exit 1; }
tail -1 gpurun_out/r02h/bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity_ok'], json.dumps(d.get('lease',{}).get('fused_with_commit',{}).get('roofline')))"
