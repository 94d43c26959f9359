set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04j
mkdir -p $O && export TMPDIR=/tmp
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d $O/sprof -o run --output-format csv -- python3 $R/scripts/stamp_bench.py > $O/sprof.log 2>&1 || { tail -20 $O/sprof.log; exit 1; }
echo done
