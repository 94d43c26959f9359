# commit / lease / fused legs of bench.py, twice
mkdir -p gpurun_out/r02q2 && export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 400 python -u bench.py --steps 50 --crc-segments 0 --no-pcie --no-cpu-baseline > gpurun_out/r02q2/bench_$i.log 2>&1 || { tail -20 gpurun_out/r02q2/bench_$i.log; exit 1; }
tail -1 gpurun_out/r02q2/bench_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['lease']; print('commit', d['roofline']['frac'], d['ms_per_step'], d['parity_ok'], 'lease', l['roofline']['frac'], l['ms_per_pass'], l['parity_ok'], 'fused', l['fused_with_commit']['roofline']['frac'], l['fused_with_commit']['parity_ok'])"
done
