#!/bin/bash
# Round 4: is the slow replay every 16 iterations (outlier_r4.sh) a count or a time (~45 s after the timed
# region starts)? The headline config with every compute task at half length (--time-scale 0.5), 36 iterations.
set -u
O=gpurun_out/outlier_scale
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
F="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph --quiet --silent -w 1 -r 36"
timeout -k 10 150 $F --time-scale 0.5 --json $O/half.json > $O/half.out 2>&1 &&
echo done >> $O/steps.log
