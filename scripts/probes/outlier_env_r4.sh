#!/bin/bash
# Round 4: the slow timed iteration every 16 replays (outlier_r4.sh) against HIP runtime batching knobs; DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (graph kernel packets built at launch instead of instantiation).
set -u
O=gpurun_out/outlier_env
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
F="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph --quiet --silent -w 1 -r 18"
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 timeout -k 10 120 $F --json $O/nocapture.json > $O/nocapture.out 2>&1 &&
echo done >> $O/steps.log
