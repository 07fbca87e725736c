#!/bin/bash
# Device timelines of the headline config (--timeline): N=1 on RCCL with the
# HIP graph, and the 8-rank FSDP config as loopback rank threads on one GPU
# (compute time-scaled). Output: gpurun_out/timeline/*.json + summaries.
set -u
mkdir -p gpurun_out/timeline
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
O=gpurun_out/timeline
timeout -k 10 120 build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 1 -r 2 \
  --quiet --silent --timeline $O/headline_n1.json --json $O/headline_n1_report.json > $O/headline_n1.log 2>&1 &&
python -m dlnetbench_amd timeline $O/headline_n1.json --check > $O/headline_n1_summary.txt 2>&1 &&
python -m dlnetbench_amd timeline $O/headline_n1.json --json > $O/headline_n1_summary.json &&
timeout -k 10 120 build/bin/fsdp llama3_8b_16_bfloat16 32 8 . --backend loopback --ranks 8 --compute gemm \
  --time-scale 0.02 -w 1 -r 2 --quiet --silent --timeline $O/fsdp_lb8.json --json $O/fsdp_lb8_report.json \
  > $O/fsdp_lb8.log 2>&1 &&
python -m dlnetbench_amd timeline $O/fsdp_lb8.json --check > $O/fsdp_lb8_summary.txt 2>&1
