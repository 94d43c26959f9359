# Round 5: where rh_crc32c_stamp_host's fixed cost goes -- the write-stamp leg under a HIP runtime +
# kernel + memory-copy trace (no counters).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r05s}
mkdir -p $O && export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 python3 -u $R/scripts/stamp_bench.py > $O/stamp_plain.log 2>&1 || { tail -20 $O/stamp_plain.log; exit 1; }
tail -1 $O/stamp_plain.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace -d $O/stamp_prof -o run --output-format csv -- python3 -u $R/scripts/stamp_bench.py > $O/stamp_prof.log 2>&1 || { tail -20 $O/stamp_prof.log; exit 1; }
ls $O/stamp_prof
