#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench, rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/abort/timeout (rc >= 124 or >= 128) stops
# the script (nothing else touches the GPU after a fault).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=$R/gpurun_out/${RUN_TAG:-run}
mkdir -p "$OUT"
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*" | tee -a "$OUT/steps.log"
  timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
  tail -5 "$OUT/$name.log"
  if [ $rc -ge 124 ]; then echo "STOP: $name rc=$rc"; exit $rc; fi
  return 0
}
rocminfo 2>/dev/null | grep -m1 -o "gfx9[0-9a-z]*" > "$OUT/arch.txt" || true
step pytest_gpu 900 python -m pytest tests -m gpu -q --timeout 300 ${PYTEST_ARGS:-}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench 900 python bench.py ${BENCH_ARGS:-}
if [ "${MICRO:-1}" = "1" ]; then step micro 600 python scripts/microbench.py --segments 32; fi
if [ "${PROFILE:-1}" = "1" ]; then
  export TMPDIR=/tmp
  step rocprof 900 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 "$R/bench.py" ${BENCH_ARGS:-}
fi
if [ "${PMC:-0}" = "1" ]; then step pmc 900 bash scripts/pmc.sh; fi
echo ALLDONE
