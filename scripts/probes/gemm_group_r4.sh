#!/bin/bash
# Round 4: tile-order group size of the one-shot GEMMs (M-tiles per group sharing B panels in L2; DLNB_GEMM_GROUP,
# default 8): fp8 one-wave-per-SIMD (v5) and bf16 8-phase (v0 = the default at these shapes), interleaved vs torch.
set -u
O=gpurun_out/ggroup
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=8192x4096x1024,8192x8192x1024,8192x4096x2048,8192x4096x14336,8192x14336x4096,8192x8192x8192,4096x4096x4096
timeout -k 10 500 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 5 --ab DLNB_GEMM_GROUP=8,4,3,6 \
  --rounds 5 --shapes $S > $O/fp8.out 2> $O/fp8.err || { echo "fp8 rc=$?" >> $O/steps.log; exit 1; }
timeout -k 10 500 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16 --variants 0 --ab DLNB_GEMM_GROUP=8,4,3,6 \
  --rounds 5 --shapes $S > $O/bf16.out 2> $O/bf16.err || { echo "bf16 rc=$?" >> $O/steps.log; exit 1; }
echo done >> $O/steps.log
