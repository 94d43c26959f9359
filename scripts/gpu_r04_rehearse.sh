# Rehearsal of bench.py's N > 1 path on a 1-GPU box: torchrun with 2 and 4 ranks sharing device 0
# over gloo (RH_BENCH_BACKEND=gloo).  Checks the line's shape and that every rank's parity holds;
# the timings are not per-GPU figures (the ranks share one GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r04n && export TMPDIR=/tmp
for n in 2; do
  RH_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
      --master-addr 127.0.0.1 --master-port $((29500 + n)) bench.py --gpus $n --steps 5 --warmup 2 \
      > $R/gpurun_out/r04n/bench_n$n.log 2>&1 || { tail -40 $R/gpurun_out/r04n/bench_n$n.log; exit 1; }
  tail -c 3000 $R/gpurun_out/r04n/bench_n$n.log
done
