# Round 5: launch fixed-cost probe under a kernel trace, then library A/B builds of the headline
# kernel (RATIS_HIP_LIB, alternating, 2 rounds) on the 1M-group config-3 launch.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05b}
mkdir -p $O && export TMPDIR=/tmp
cd /tmp
if [ "${PROBE:-1}" = 1 ]; then
timeout -k 10 120 rocprofv3 --kernel-trace -d $O/probe_prof -o run --output-format csv -- $R/scripts/ablation/launch_probe > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
grep probe $O/probe.log
fi
for r in 1 2; do
for lib in $R/ratis_amd/lib/libratis_hip.so $R/ratis_amd/lib/ab/*.so; do
  tag=$(basename $lib .so)
  RATIS_HIP_LIB=$lib timeout -k 10 200 python3 -u $R/scripts/commit_sweep.py --sizes ${SIZES:-1000000} --rounds 5 > $O/${tag}_$r.log 2>&1 || { tail -20 $O/${tag}_$r.log; exit 1; }
  echo "== $tag $r: $(grep us_per_launch $O/${tag}_$r.log | python3 -c 'import sys,json; print([ (d["groups"], d["us_per_launch"]) for d in map(json.loads, sys.stdin)])')"
done
done
