#!/bin/bash
# Round 5: the headline's occasional 2x-slow last reduce-scatter (barrier 0.36 vs 0.19 ms): full-scale FSDP, 12
# iterations per run, host_wait tight polling forever (0) vs backoff after 50 us (default), alternating.
set -u
O=${O:-gpurun_out/rs_spike}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
H="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph --quiet --silent -w 2 -r 12"
for rep in a b; do
  for t in 0 50; do
    echo "t$t$rep start $(date +%s)" >> $O/steps.log
    DLNB_HOST_WAIT_TIGHT_US=$t timeout -k 10 200 $H --json $O/t${t}_$rep.json > $O/t${t}_$rep.log 2>&1 || { echo "rc=$?" >> $O/steps.log; exit 1; }
  done
done
echo done >> $O/steps.log
