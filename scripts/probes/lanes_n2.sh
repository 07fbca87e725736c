#!/bin/bash
# Round 5: the multi-rank lane-graph path rehearsed on one GPU - 2 processes of the FSDP headline step (llama3_8b,
# U = 32, F = 2, --time-scale 0.05) over the xgmi kernels, each rank's deadline grid on 96 CUs (--comm-cus 160: the
# two grids fit side by side with 64 CUs for the collectives), no slicing; lane graphs forced despite the shared
# device (DLNB_LANE_SHARED=1) against the single graph. Every wait is bounded (gates 5 s, xgmi 60 s).
set -u
O=${O:-gpurun_out/lanes_n2}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5 DLNB_XGMI_TIMEOUT_S=60 DLNB_GEMM_SLICE_US=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run2() {  # name port env...
  local n=$1 port=$2; shift 2
  echo "$n start $(date +%s)" >> $O/steps.log
  local pids=()
  for r in 0 1; do
    env "$@" RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      timeout -k 10 150 build/bin/fsdp llama3_8b_16_bfloat16 32 2 . --backend xgmi --devices 0,0 --comm-cus 160 --rccl-max-ctas 8 \
      --compute gemm --graph -w 3 -r 12 --time-scale 0.05 --quiet --silent --json $O/$n.r$r.json > $O/$n.r$r.log 2>&1 &
    pids+=($!)
  done
  local rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "$n rc=$rc" >> $O/steps.log
  return $rc
}
run2 single 29611 DLNB_LANE_GRAPHS=0 && run2 lanes 29621 DLNB_LANE_SHARED=1 && run2 single_b 29631 DLNB_LANE_GRAPHS=0 \
  && run2 lanes_b 29641 DLNB_LANE_SHARED=1
