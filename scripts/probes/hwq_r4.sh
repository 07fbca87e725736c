#!/bin/bash
# Round 4: the C5 step (graph, event edges) with more hardware queues per process (GPU_MAX_HW_QUEUES; the box
# default is 4): the graph executor rotates the backward GEMMs over its queues and queued one behind an all-reduce
# on the comm chain's queue every 4 buckets (profiles/absorb_r4.md). Timing + chain_capped per setting, a trace at
# 8, and the headline at 8 vs 4.
set -u
O=gpurun_out/hwq
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 5 -r 30 --quiet --silent"
for q in 4 5 6 8 12 4; do
  env GPU_MAX_HW_QUEUES=$q timeout -k 10 120 $C5 --json $O/c5_q$q.json > $O/c5_q$q.log 2>&1 || { echo "rc=$? q=$q" >> $O/steps.log; exit 1; }
  echo "q=$q ok" >> $O/steps.log
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
GPU_MAX_HW_QUEUES=8 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_q8 -o c5 -- $C5 \
  > $O/trace_q8.log 2>&1 || { echo "trace rc=$?" >> $O/steps.log; exit 1; }
unset DLNB_NO_TORCH
for q in 8 4; do
  env GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0 \
    > $O/head_q$q.json 2> $O/head_q$q.err || { echo "head rc=$? q=$q" >> $O/steps.log; exit 1; }
done
echo done >> $O/steps.log
