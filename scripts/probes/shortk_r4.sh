#!/bin/bash
# Round 4: the fp8 short-K shape (8192 x 4096 x 1024: 8 K-tiles, 512 square tiles = 2 per CU on the streaming
# kernel) at 0.89-0.90x _scaled_mm. A/B of the tile width (DLNB_GEMM_NARROW_NF: 8 = square, 4 = 256 x 128: 1024
# tiles, half the epilogue per tile) and the stall PMC of ours vs the vendor at that shape.
set -u
O=gpurun_out/shortk
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 0 --ab DLNB_GEMM_NARROW_NF=8,4 \
  --rounds 7 --shapes 8192x4096x1024,8192x8192x1024,4096x4096x1024,8192x4096x2048 > $O/ab.out 2> $O/ab.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES GRBM_GUI_ACTIVE"
for p in 1 2; do
  if [ $p = 1 ]; then C=$P1; else C=$P2; fi
  timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$p -o g -- python3 -m dlnetbench_amd.tools.gemm_bench \
    --dtype fp8 --variants 5 --shapes 8192x4096x1024 --rounds 2 --iters 10 > $O/pmc_$p.log 2>&1 || exit $?
done
echo done > $O/done.txt
