#!/bin/bash
# Device timeline of the comm-bound C5 step (vit_h_32_float8 DP, 8 buckets,
# HIP graph) at N = 1, even and geometric (0.7) buckets.
set -u
mkdir -p gpurun_out/c5tl
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
O=gpurun_out/c5tl
timeout -k 10 120 build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 5 -r 20 --quiet --silent \
  --timeline $O/even.json --timeline-iters 3 --json $O/even_report.json > $O/even.log 2>&1 &&
timeout -k 10 120 build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 5 -r 20 --quiet --silent \
  --dp-bucket-ratio 0.7 --timeline $O/geo.json --timeline-iters 3 --json $O/geo_report.json > $O/geo.log 2>&1 &&
python -m dlnetbench_amd timeline $O/even.json --check > $O/even_summary.txt 2>&1 &&
python -m dlnetbench_amd timeline $O/geo.json --check > $O/geo_summary.txt 2>&1
