#!/bin/bash
# Round 5: lanes vs the single graph for a pipeline WITH tensor parallelism (hybrid_3d S=2 mb=4 T=2: PP P2P on
# their own lanes, TP all-reduces on the compute lane), 4 ranks on one GPU over xgmi, two time scales.
# (lanes_tp_n2.sh measured S=1 only: no P2P, where lanes only add overhead.)
set -u
O=${O:-gpurun_out/lanes_tp_pp_n4}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=10 DLNB_XGMI_TIMEOUT_S=30 DLNB_GEMM_SLICE_US=0
run4() {  # name port scale env...
  local n=$1 port=$2 scale=$3; shift 3
  echo "$n start $(date +%s)" >> $O/steps.log
  local pids=()
  for r in 0 1 2 3; do
    env "$@" RANK=$r WORLD_SIZE=4 LOCAL_RANK=$r LOCAL_WORLD_SIZE=4 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      DLNB_STORE_PORT=$((port + 5)) timeout -k 10 120 build/bin/hybrid_3d llama3_8b_16_bfloat16 2 4 2 . --backend xgmi \
      --devices 0,0,0,0 --comm-cus 160 --rccl-max-ctas 8 --compute gemm --graph -w 3 -r 8 --time-scale $scale \
      --json $O/$n.r$r.json > $O/$n.r$r.log 2>&1 &
    pids+=($!)
  done
  local rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "$n rc=$rc $(date +%s)" >> $O/steps.log
  return $rc
}
run4 s05_lanes 29811 0.05 DLNB_LANE_SHARED=1 DLNB_LANE_GRAPHS=2 && run4 s05_single 29821 0.05 DLNB_LANE_GRAPHS=0 \
  && run4 s20_lanes 29831 0.2 DLNB_LANE_SHARED=1 DLNB_LANE_GRAPHS=2 && run4 s20_single 29841 0.2 DLNB_LANE_GRAPHS=0
