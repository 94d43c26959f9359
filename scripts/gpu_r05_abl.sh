# Round 5: headline-kernel ablations at 1M groups (bits / min column / one tier / trivial arithmetic).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05k}
mkdir -p $O && export TMPDIR=/tmp
cd $R
run() {
  tag=$1; shift
  timeout -k 10 200 python3 -u scripts/commit_sweep.py --sizes 1000000 --rounds 5 "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  echo "$tag $(grep us_per_launch $O/$tag.log | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["us_per_launch"], d["alg_TBps"])')"
}
for r in 1 2; do
run base_$r
run nobits_$r --no-bits
run nomin_$r --no-min
run stable_$r --tiers stable
run joint_$r --tiers joint
RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_noeval.so run noeval_$r
RATIS_HIP_LIB=$R/ratis_amd/lib/ab/libratis_hip_noeval.so run noeval_stable_$r --tiers stable
done
