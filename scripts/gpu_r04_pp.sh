# Round 4: packed CRC kernel with the step loop over two register sets (no copy of the prefetched
# chunk) -- CRC / read-path GPU tests on the A/B build, then the ragged read launch under a kernel
# trace, shipped build and A/B build alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04pp}
mkdir -p $O && export TMPDIR=/tmp
AB=$R/ratis_amd/lib/ab/libratis_hip_${2:-pp}.so
RATIS_HIP_LIB=$AB timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py > $O/pytest_ab.log 2>&1 || { tail -60 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
n=0
for lib in $R/ratis_amd/lib/libratis_hip.so $AB $R/ratis_amd/lib/libratis_hip.so $AB; do
  n=$((n + 1)); tag=$(basename $lib .so)_$n
  cd /tmp && RATIS_HIP_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/rr_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what ragged_read --segments 128 --iters 6 > $O/rr_$tag.log 2>&1 || { tail -5 $O/rr_$tag.log; exit 1; }
  cd $R && python3 - $O/rr_$tag $tag <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0])))
pick = {r["Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[-40:]: round(float(r["AverageNs"]) / 1000, 1)
        for r in rows if any(k in r["Name"] for k in ("crc_pack", "piece_guess", "piece_walk", "crc_frames"))}
print(sys.argv[2], pick)
PY
done
