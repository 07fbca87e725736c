#!/bin/bash
# Round 5: diagnose the 2-process shared-GPU lane run (lanes_n2.sh): short runs with logs, per-rank timeouts.
set -u
O=${O:-gpurun_out/lanes_n2b}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5 DLNB_XGMI_TIMEOUT_S=20 DLNB_GEMM_SLICE_US=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
run1() {  # name env...
  local n=$1; shift
  echo "$n start $(date +%s)" >> $O/steps.log
  env "$@" timeout -k 10 60 build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --comm-cus 160 \
    --compute gemm --graph -w 2 -r 4 --time-scale 0.05 --json $O/$n.json > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/steps.log; return $rc
}
run2() {  # name port env...
  local n=$1 port=$2; shift 2
  echo "$n start $(date +%s)" >> $O/steps.log
  local pids=()
  for r in 0 1; do
    env "$@" RANK=$r WORLD_SIZE=2 LOCAL_RANK=$r LOCAL_WORLD_SIZE=2 MASTER_ADDR=127.0.0.1 MASTER_PORT=$port \
      timeout -k 10 75 build/bin/fsdp llama3_8b_16_bfloat16 32 2 . --backend xgmi --devices 0,0 --comm-cus 160 --rccl-max-ctas 8 \
      --compute gemm --graph -w 3 -r 12 --time-scale 0.05 ${EXTRA:-} --json $O/$n.r$r.json > $O/$n.r$r.log 2>&1 &
    pids+=($!)
  done
  local rc=0
  for p in "${pids[@]}"; do wait $p || rc=$?; done
  echo "$n rc=$rc" >> $O/steps.log
  return $rc
}
run2 single 29671 DLNB_LANE_GRAPHS=0 && run2 lanes 29661 DLNB_LANE_SHARED=1 && run2 lanes_noalt 29681 DLNB_LANE_SHARED=1 DLNB_LANE_ALTERNATE=0 \
  && run2 lanes_noprearm 29691 DLNB_LANE_SHARED=1 DLNB_PREARM=0 && run2 lanes_noprog 29701 DLNB_LANE_SHARED=1 DLNB_LANE_GRAPHS=2 DLNB_COMPUTE_PROGRAMS=0 \
  && run2 single_b 29711 DLNB_LANE_GRAPHS=0 && run2 lanes_b 29721 DLNB_LANE_SHARED=1 && EXTRA=--timeline run2 lanes_timeline 29731 DLNB_LANE_SHARED=1
