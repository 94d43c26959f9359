# CRC leg with the longer warmup, twice, plus its kernel trace once
mkdir -p gpurun_out/r02w && export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 400 python -u bench.py --steps 10 --no-lease --no-pcie --no-cpu-baseline --ragged-segments 0 > gpurun_out/r02w/bench_$i.log 2>&1 || { tail -20 gpurun_out/r02w/bench_$i.log; exit 1; }
tail -1 gpurun_out/r02w/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['crc32c']; print('crc', c['GBps'], c['roofline']['frac'], c['ms_per_pass'], c['parity_ok'], 'read', c['read_path']['read_launch_GBps'])"
done
