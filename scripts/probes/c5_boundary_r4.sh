#!/bin/bash
# Round 4: the C5 comm-bound step (dp vit_h_32_float8, 8 buckets, HIP graph, N = 1) on the device timeline with
# the graph launch edges, pre-armed loop (default) and the round-4 loop (DLNB_PREARM=0).
set -u
O=gpurun_out/c5b
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_TIMELINE_EDGES=1
F="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 5 -r 6 --quiet --silent --timeline-iters 6"
timeout -k 10 120 $F --timeline $O/prearm.json --json $O/prearm_report.json > $O/prearm.out 2>&1 &&
DLNB_PREARM=0 timeout -k 10 120 $F --timeline $O/old.json --json $O/old_report.json > $O/old.out 2>&1 &&
timeout -k 10 60 python -m dlnetbench_amd timeline $O/prearm.json > $O/prearm_sum.txt 2>&1 &&
timeout -k 10 60 python -m dlnetbench_amd timeline $O/old.json > $O/old_sum.txt 2>&1 &&
echo done >> $O/steps.log
