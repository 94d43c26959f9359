# Round 5: resident-table hasLease pass A/B (scripts/table_lease_bench.py per library, alternating,
# 2 rounds), then the shipped library under a kernel trace.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05tl}
mkdir -p $O && export TMPDIR=/tmp
cd $R
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $(ls $R/ratis_amd/lib/ab/*.so 2>/dev/null); do
  tag=$(basename $lib .so)_$r
  RATIS_HIP_LIB=$lib timeout -k 10 300 python3 -u scripts/table_lease_bench.py > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo $tag $(grep '^{' $O/$tag.log | tail -1)
done
done
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -u $R/scripts/table_lease_bench.py > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep -h "table_lease_kernel" $O/prof/*/run_kernel_stats.csv $O/prof/run_kernel_stats.csv 2>/dev/null | head -5
