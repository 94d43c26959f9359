# Resident table: parity tests + delta-streaming stage timing
mkdir -p gpurun_out/r02i && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_table.py > gpurun_out/r02i/pytest.log 2>&1 || { tail -40 gpurun_out/r02i/pytest.log; exit 1; }
tail -3 gpurun_out/r02i/pytest.log
timeout -k 10 200 python -u scripts/pcie_bench.py > gpurun_out/r02i/pcie.log 2>&1 || { tail -20 gpurun_out/r02i/pcie.log; exit 1; }
cat gpurun_out/r02i/pcie.log
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/r02i/prof -o run --output-format csv -- python3 scripts/pcie_bench.py --steps 10 > gpurun_out/r02i/prof.log 2>&1
