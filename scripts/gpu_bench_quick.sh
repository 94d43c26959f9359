# commit / lease / fused legs of bench.py: graph-captured timed loops vs stream launches
mkdir -p gpurun_out/r02q3 && export TMPDIR=/tmp
for mode in graph stream graph stream; do
extra=""; [ $mode = stream ] && extra="--no-graph"
timeout -k 10 400 python -u bench.py --steps 50 --crc-segments 0 --no-pcie --no-cpu-baseline $extra > gpurun_out/r02q3/bench_$mode.log 2>&1 || { tail -20 gpurun_out/r02q3/bench_$mode.log; exit 1; }
tail -1 gpurun_out/r02q3/bench_$mode.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); l=d['lease']; print('$mode', d['config']['timed_launches'], 'commit', d['roofline']['frac'], d['ms_per_step'], d['parity_ok'], 'lease', l['roofline']['frac'], l['ms_per_pass'], l['parity_ok'], 'fused', l['fused_with_commit']['roofline']['frac'], l['fused_with_commit']['parity_ok'])"
done
