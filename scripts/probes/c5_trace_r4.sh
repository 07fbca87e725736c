#!/bin/bash
# Round 4: what the comm-bound C5 step's exposed tail (the last bucket's all-reduce after the backward) is made
# of at N = 1: kernel + memory-copy trace of the even-bucket step (which kernels / copies RCCL issues for a
# 1-rank all-reduce of 158 MB, and how long each takes), then the device timeline.
set -u
O=gpurun_out/c5tr
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/trace -o c5 -- \
  build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 3 -r 5 --quiet --silent \
  --json $O/trace_report.json > $O/trace.log 2>&1 &&
timeout -k 10 120 build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 5 -r 20 --quiet --silent \
  --timeline $O/even.json --timeline-iters 3 --json $O/even_report.json > $O/even.log 2>&1 &&
python -m dlnetbench_amd timeline $O/even.json --check > $O/even_summary.txt 2>&1
