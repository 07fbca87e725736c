#!/bin/bash
# Pipeline schedules at S = 2 on two processes sharing ONE MI355X (xgmi backend):
# hybrid_2d llama3_8b, mb = 8, --compute sleep, compute scaled by 0.25. Two
# ranks x few streams stay within the hardware queues (interleaved_xgmi_r1.md),
# so the iteration times show the schedules' bubbles. Stops at the first failure.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=30 DLNB_TIMEOUT=100
step() {  # name extra-args...
  local name=$1; shift
  timeout -k 10 150 python -m dlnetbench_amd.utils.launch -n 2 --timeout 140 build/bin/hybrid_2d llama3_8b_16_bfloat16 \
    2 8 . "$@" -w 1 -r 3 --backend xgmi -d 0,0 --compute sleep --time-scale 0.25 --no-topology --quiet \
    --json gpurun_out/x2_$name.json > gpurun_out/x2_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/x2_steps.log
  return $rc
}
step gpipe --pp-schedule gpipe && step 1f1b --pp-schedule 1f1b && step dualpipe --pp-schedule dualpipe
