#!/bin/bash
# Round 5: lane graphs without a compute program for long-task strategies (DLNB_LANE_MIN_TASK_US): one-rank hybrids
# (llama3_8b, --time-scale 0.05) lanes vs single graph, and the 2-rank pipeline on one GPU with the default rule.
set -u
O=${O:-gpurun_out/lanes_hyb}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run1() {  # name binary params... (env LG)
  local n=$1; shift
  echo "$n start $(date +%s)" >> $O/steps.log
  env DLNB_LANE_GRAPHS=${LG:-1} timeout -k 10 120 "$@" . --backend rccl --compute gemm --graph -w 3 -r 10 --time-scale 0.05 \
    --quiet --silent --json $O/$n.json > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/steps.log; return $rc
}
run1 cp_lanes build/bin/hybrid_cp llama3_8b_16_bfloat16 1 && LG=0 run1 cp_single build/bin/hybrid_cp llama3_8b_16_bfloat16 1 \
  && run1 h3_lanes build/bin/hybrid_3d llama3_8b_16_bfloat16 1 4 1 && LG=0 run1 h3_single build/bin/hybrid_3d llama3_8b_16_bfloat16 1 4 1 \
  && run1 h2_lanes build/bin/hybrid_2d llama3_8b_16_bfloat16 1 4 && LG=0 run1 h2_single build/bin/hybrid_2d llama3_8b_16_bfloat16 1 4 \
  && run1 moe_lanes build/bin/hybrid_3d_moe mixtral_8x7b_16_bfloat16 1 4 1 \
  && run1 cp_lanes2 build/bin/hybrid_cp llama3_8b_16_bfloat16 1 && LG=0 run1 cp_single2 build/bin/hybrid_cp llama3_8b_16_bfloat16 1
