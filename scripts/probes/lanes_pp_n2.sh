#!/bin/bash
# Round 5: lane graphs for the pipeline hybrids, rehearsed with 2 processes on one GPU (xgmi): hybrid_3d llama3_8b
# S = 2, mb = 4 / 8, T = 1 at --time-scale 0.05; single graph vs lanes with one launch per task
# (DLNB_LANE_GRAPHS=2: the pipeline has no compute program). Collectives capped at 8 CTAs, grids on 96 CUs.
set -u
O=${O:-gpurun_out/lanes_pp_n2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5 DLNB_XGMI_TIMEOUT_S=20 DLNB_GEMM_SLICE_US=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run2() {  # name port mb env...
  local n=$1 port=$2 mb=$3; shift 3
  echo "$n start $(date +%s)" >> $O/steps.log
  local pids=()
  for r in 0 1; do
    env "$@" RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      timeout -k 10 90 build/bin/hybrid_3d llama3_8b_16_bfloat16 2 $mb 1 . --backend xgmi --devices 0,0 --comm-cus 160 \
      --rccl-max-ctas 8 --compute gemm --graph -w 3 -r 10 --time-scale 0.05 --json $O/$n.r$r.json > $O/$n.r$r.log 2>&1 &
    pids+=($!)
  done
  local rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "$n rc=$rc" >> $O/steps.log
  return $rc
}
run2 single4 29811 4 DLNB_LANE_GRAPHS=0 && run2 lanes4 29821 4 DLNB_LANE_SHARED=1 \
  && run2 single8 29831 8 DLNB_LANE_GRAPHS=0 && run2 lanes8 29841 8 DLNB_LANE_SHARED=1 DLNB_LANE_GRAPHS=2 \
  && run2 single4b 29851 4 DLNB_LANE_GRAPHS=0 && run2 lanes4b 29861 4 DLNB_LANE_SHARED=1 DLNB_LANE_GRAPHS=2
