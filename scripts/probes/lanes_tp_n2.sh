#!/bin/bash
# Round 5: lane graphs with TP collectives on the compute lane: hybrid_3d S=1 mb=4 T=2 (2 ranks on one GPU, xgmi),
# lanes (long tasks, no program) vs the single graph; and hybrid_2d S=2 mb=4 the same way.
set -u
O=${O:-gpurun_out/lanes_tp_n2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5 DLNB_XGMI_TIMEOUT_S=20 DLNB_GEMM_SLICE_US=0
run2() {  # name port binary params... -- env
  local n=$1 port=$2 bin=$3 params=$4; shift 4
  echo "$n start $(date +%s)" >> $O/steps.log
  local pids=()
  for r in 0 1; do
    env "$@" RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      timeout -k 10 90 build/bin/$bin llama3_8b_16_bfloat16 $params . --backend xgmi --devices 0,0 --comm-cus 160 \
      --rccl-max-ctas 8 --compute gemm --graph -w 3 -r 10 --time-scale 0.05 --json $O/$n.r$r.json > $O/$n.r$r.log 2>&1 &
    pids+=($!)
  done
  local rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "$n rc=$rc" >> $O/steps.log
  return $rc
}
run2 tp_lanes 29911 hybrid_3d "1 4 2" DLNB_LANE_SHARED=1 && run2 tp_single 29921 hybrid_3d "1 4 2" DLNB_LANE_GRAPHS=0 \
  && run2 h2_lanes 29931 hybrid_2d "2 4" DLNB_LANE_SHARED=1 && run2 h2_single 29941 hybrid_2d "2 4" DLNB_LANE_GRAPHS=0
