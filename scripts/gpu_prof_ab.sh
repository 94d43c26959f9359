# kernel-trace split of one CRC shape under two library builds
mkdir -p gpurun_out/pab && export TMPDIR=/tmp
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_q12_16.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/pab/$tag -o run --output-format csv -- python3 scripts/prof_kernels.py --what crcshape --frame-size 256 --segments 96 --iters 5 > gpurun_out/pab/$tag.log 2>&1 || { tail -5 gpurun_out/pab/$tag.log; exit 1; }
  echo "== $tag"; python scripts/prof_summary.py $(find gpurun_out/pab/$tag -name '*kernel_trace.csv' | head -1) --top 8 | grep crc
done
