# Round 4: direct event lists + the packed CRC kernel folding chunk 0 in its steps -- GPU suite,
# the table leg at 100 / 10 / 1 / 0.1 % dirty under a kernel trace, and the ragged read A/B against
# the chunk-0-pass build (bench leg, kernel trace, FETCH_SIZE).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04s}
mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_table_events.py tests/test_gpu_table.py tests/test_gpu_node.py tests/test_gpu_crc.py tests/test_gpu_segread.py > $O/pytest_first.log 2>&1 || { tail -60 $O/pytest_first.log; exit 1; }
tail -1 $O/pytest_first.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tprof -o run --output-format csv -- python3 $R/scripts/table_bench.py --reps 6 --fracs 1.0,0.1,0.01,0.001 > $O/tb.log 2>&1 || { tail -30 $O/tb.log; exit 1; }
cd $R && python - $O/tb.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])["table_commit"]
for k, v in d.items():
    if isinstance(v, dict):
        print(k, "eval", v["ms_evaluation"], "list", v["list_mode"], "hm", v["host_mapped"], "dev", v["device"], "auto", v["auto"], "frac", v["roofline"]["frac"], "agree", v["sinks_agree"], "adv", v["advanced"])
PY
for lib in ratis_amd/lib/libratis_hip.so ratis_amd/lib/ab/libratis_hip_c0pass.so; do
  tag=$(basename $lib .so)
  cd /tmp && RATIS_HIP_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/rrprof_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 6 > $O/rrprof_$tag.log 2>&1 || { tail -5 $O/rrprof_$tag.log; exit 1; }
  RATIS_HIP_LIB=$R/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/rrpmc_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 64 --iters 4 > $O/rrpmc_$tag.log 2>&1 || { tail -5 $O/rrpmc_$tag.log; exit 1; }
  cd $R
done
echo done
