# Packed CRC kernel: A/B against the length-class split (and packed-for-all) on one box
mkdir -p gpurun_out/ab && export TMPDIR=/tmp
SEGS=${SEGS:-128} SECTIONS=crc,crcshape,ragread,readc5 bash scripts/gpu_ab.sh > gpurun_out/ab/run.txt 2>&1 || { tail -30 gpurun_out/ab/run.txt; exit 1; }
python scripts/ab_table.py
