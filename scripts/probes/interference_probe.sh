#!/bin/bash
# Interference on one MI355X: the headline FSDP config (llama3_8b U=32,
# fixed-work gemm-work compute, time-scaled 0.25, HIP graph) as the victim,
# the comm-bound ViT-H DP step (1.26 GB of all-reduce every 7 ms + deadline
# GEMMs, HIP graph, --loop) as the aggressor, both 1-rank RCCL jobs on GPU 0.
set -u
mkdir -p gpurun_out/interference
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
timeout -k 10 400 python -m dlnetbench_amd interference \
  --victim "fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm-work --graph -w 1 -r 3 --time-scale 0.25" \
  --aggressor "dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph" --warm-s 8 --timeout 150 \
  --json gpurun_out/interference/fsdp_vs_dp_same_gpu.json > gpurun_out/interference/log.txt 2>&1
