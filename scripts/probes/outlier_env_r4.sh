#!/bin/bash
# Round 4: the slow timed iteration every 16 replays (outlier_r4.sh) against HIP runtime batching knobs.
set -u
O=gpurun_out/outlier_env
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
F="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph --quiet --silent -w 1 -r 18"
DEBUG_CLR_BATCH_CPU_SYNC_SIZE=1024 timeout -k 10 120 $F --json $O/cpusync.json > $O/cpusync.out 2>&1 &&
DEBUG_CLR_MAX_BATCH_SIZE=1024 timeout -k 10 120 $F --json $O/maxbatch.json > $O/maxbatch.out 2>&1 &&
DEBUG_HIP_GRAPH_BATCH_SIZE=1024 timeout -k 10 120 $F --json $O/graphbatch.json > $O/graphbatch.out 2>&1 &&
echo done >> $O/steps.log
