mkdir -p gpurun_out/r02e && export TMPDIR=/tmp
for mf in 2048 512; do
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d gpurun_out/r02e/a$mf -o run --output-format csv -- python3 scripts/prof_kernels.py --what ragged --segments 64 --iters 2 --max-frame $mf > gpurun_out/r02e/a$mf.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_INSTS_SMEM -d gpurun_out/r02e/b$mf -o run --output-format csv -- python3 scripts/prof_kernels.py --what ragged --segments 64 --iters 2 --max-frame $mf > gpurun_out/r02e/b$mf.log 2>&1 || exit 1
done
echo done
