#!/bin/bash
# A/B builds of libratis_hip for tuning (never loaded by the product, tests or bench.py):
#   ratis_amd/lib/ab/libratis_hip_<name>.so, selected with RATIS_HIP_LIB=... by scripts.
# Usage: scripts/ab_build.sh <name> "<extra hipcc flags>"
set -e
cd "$(dirname "$0")/../ratis_amd/csrc"
name=$1; flags=$2
out=../lib/ab; obj=../../build/ab_$name
mkdir -p $out $obj
for f in commit crc32c segment segread lease table; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden $flags -c $f.hip -o $obj/$f.o &
done
for f in rh_api groups; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -fvisibility=hidden $flags -x hip -c $f.cpp -o $obj/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libratis_hip_$name.so $obj/*.o
echo built $out/libratis_hip_$name.so
