# Round 4: CRC folds with gfx950's 3-input XOR (v_bitop3: a word's four lookups and the next word
# joined in two ops) + the packed kernel's two register sets -- CRC / read-path GPU tests on the A/B
# build, then kernel traces of the ragged read launch, the config-5 window kernel and the frame-API
# packed kernel, shipped build and A/B build alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04x3}
mkdir -p $O && export TMPDIR=/tmp
AB=$R/ratis_amd/lib/ab/libratis_hip_${2:-x3}.so
AB2=$R/ratis_amd/lib/ab/libratis_hip_${3:-pp}.so
RATIS_HIP_LIB=$AB timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_crc.py tests/test_gpu_segread.py > $O/pytest_ab.log 2>&1 || { tail -60 $O/pytest_ab.log; exit 1; }
tail -1 $O/pytest_ab.log
n=0
for lib in $R/ratis_amd/lib/libratis_hip.so $AB $AB2 $R/ratis_amd/lib/libratis_hip.so $AB $AB2; do
  n=$((n + 1)); tag=$(basename $lib .so)_$n
  for w in "ragged_read --segments 128" "crc --segments 32" "crcragged --segments 64"; do
    wt=$(echo $w | cut -d' ' -f1)
    cd /tmp && RATIS_HIP_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats -d $O/${wt}_$tag -o run --output-format csv -- python3 $R/scripts/prof_kernels.py --what $w --iters 6 > $O/${wt}_$tag.log 2>&1 || { tail -5 $O/${wt}_$tag.log; exit 1; }
    cd $R && python3 - $O/${wt}_$tag "$wt $tag" <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0])))
pick = {r["Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[-34:]: round(float(r["AverageNs"]) / 1000, 1)
        for r in rows if any(k in r["Name"] for k in ("crc_pack", "piece_guess", "piece_walk", "crc_frames"))}
print(sys.argv[2], pick)
PY
  done
done
