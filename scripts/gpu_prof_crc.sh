# kernel split of the CRC launch: config 5 frames and the ragged read launch (rocprofv3 kernel trace)
mkdir -p gpurun_out/r02pc && export TMPDIR=/tmp
for what in ${WHATS:-crc ragged_read}; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r02pc/$what -o run --output-format csv -- python3 scripts/prof_kernels.py --what $what --segments 256 --iters 5 > gpurun_out/r02pc/$what.log 2>&1 || { tail -30 gpurun_out/r02pc/$what.log; exit 1; }
python scripts/prof_summary.py $(find gpurun_out/r02pc/$what -name '*kernel_trace.csv' | head -1) --out gpurun_out/r02pc/$what.md --top 12 > /dev/null
grep -v "at::native" gpurun_out/r02pc/$what.md | head -14
done
