#!/bin/bash
# Round 5: long replay runs of the lane-graph paths (gate tags, program epochs, alternating sets over many
# replays): C5 1000 iterations, the headline at 0.05x 300, one-rank hybrid_3d (lanes without a program) 200.
set -u
O=${O:-gpurun_out/soak}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run1() {
  local n=$1; shift
  echo "$n start $(date +%s)" >> $O/steps.log
  "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/steps.log; return $rc
}
run1 c5 timeout -k 10 120 build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 5 -r 1000 --quiet --silent --json $O/c5.json \
  && run1 head timeout -k 10 150 build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 3 -r 300 --time-scale 0.05 --quiet --silent --json $O/head.json \
  && run1 h3 timeout -k 10 150 build/bin/hybrid_3d llama3_8b_16_bfloat16 1 4 1 . --backend rccl --compute gemm --graph -w 3 -r 200 --time-scale 0.05 --quiet --silent --json $O/h3.json
