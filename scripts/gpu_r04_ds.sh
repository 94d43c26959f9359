# Round 4: delta streaming per event sink (AUTO / HOST_MAPPED / DEVICE), same process, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04ds}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/ds_bench.py > $O/ds.log 2>&1 || { tail -30 $O/ds.log; exit 1; }
grep -v "^{" $O/ds.log | tail -4
