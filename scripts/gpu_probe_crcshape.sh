# CRC cost vs frame shape, and the ragged read launch's kernel split
mkdir -p gpurun_out/r02p && export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/microbench.py --only crcshape --segments 64 --rounds 3 > gpurun_out/r02p/micro.log 2>&1 || { tail -30 gpurun_out/r02p/micro.log; exit 1; }
cat gpurun_out/r02p/micro.log | grep kernel
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02p/prof -o run --output-format csv -- python3 scripts/prof_kernels.py --what ragged_read --segments 256 --iters 5 > gpurun_out/r02p/prof.log 2>&1 || { tail -30 gpurun_out/r02p/prof.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/r02p/prof -name '*kernel_trace.csv' | head -1) --out gpurun_out/r02p/dispatch.md
cat gpurun_out/r02p/dispatch.md
