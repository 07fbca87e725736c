#!/bin/bash
# Round 4: every 20-step N = 1 headline run had one iteration ~1 ms slower, always timed iteration 16 whatever the
# warm-up count (the device-side timers of that iteration are normal: the time is lost on the host side of the
# replay). Periodicity over 40 iterations, and the HIP runtime's signal pool as the suspect (ROC_SIGNAL_POOL_SIZE).
set -u
O=gpurun_out/outlier
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
F="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph --quiet --silent -w 1 -r 40"
timeout -k 10 200 $F --json $O/r40.json > $O/r40.out 2>&1 &&
ROC_SIGNAL_POOL_SIZE=4096 timeout -k 10 200 $F --json $O/r40_pool.json > $O/r40_pool.out 2>&1 &&
echo done >> $O/steps.log
