#!/bin/bash
# fp8 one-wave-per-SIMD GEMM: one block per tile (DLNB_GEMM_FP8_STREAM=0) vs the streaming persistent kernel (1).
for s in 0 1; do
  echo "STREAM=$s"
  DLNB_GEMM_FP8_STREAM=$s timeout -k 10 150 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 5 \
    --shapes 8192x8192x8192,8192x14336x4096,8192x5120x1280,8192x1280x5120 || exit 1
done
