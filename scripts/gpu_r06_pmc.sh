# Round 6: PMC passes at HEAD (one rocprofv3 run per counter group, kernel-trace only, no other
# trace domain) of every kernel whose roofline carries `traffic`: the headline commit kernel, config
# 5's CRC verify, the framing walk, the lease kernel, the resident-table evaluation (100 % dirty) and
# the ragged read launch.  Summarised by scripts/pmc_summary.py (+ pmc_ragged.py) into
# gpurun_out/<tag>/pmc_traffic.json, committed as profiles/r06/pmc_traffic.json.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r06pmc}
mkdir -p $O/pmc && export TMPDIR=/tmp
cd /tmp
run() { local name=$1 ctrs=$2; shift 2
  timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctrs -d "$O/pmc/$name" -o run --output-format csv -- python3 $R/scripts/prof_kernels.py "$@" > "$O/$name.log" 2>&1
  local rc=$?; echo "$name rc=$rc"; if [ $rc -ne 0 ]; then tail -20 "$O/$name.log"; exit $rc; fi; }
S="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
for w in "commit --iters 8" "crc --segments 32 --iters 5" "lease --iters 8" "table --iters 6"; do
  t=${w%% *}
  run ${t}_a "$S" --what $w
  run ${t}_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what $w
  run ${t}_w "WRITE_SIZE" --what $w
done
run framing_a "$S" --what framing --segments 64
run framing_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what framing --segments 64
run framing_w "WRITE_SIZE" --what framing --segments 64
run rr_b "FETCH_SIZE GRBM_GUI_ACTIVE" --what ragged_read --segments 64 --iters 4
run rr_w "WRITE_SIZE" --what ragged_read --segments 64 --iters 4
cp $O/rr_b.log $O/pmc/rr_b.log
python3 $R/scripts/pmc_summary.py $O/pmc --out $O/pmc_traffic.json > /dev/null && \
python3 $R/scripts/pmc_ragged.py $O/pmc --iters 4 --merge $O/pmc_traffic.json > $O/ragged.txt && echo PMCDONE
