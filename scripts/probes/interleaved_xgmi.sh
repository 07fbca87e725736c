#!/bin/bash
# Diagnose pipeline schedules on 4 ranks sharing one GPU over xgmi (each step time-limited; stop at the first failure).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=20 DLNB_TIMEOUT=45
step() {  # name extra-args...
  local name=$1; shift
  timeout -k 10 90 python -m dlnetbench_amd.utils.launch -n 4 --timeout 80 build/bin/hybrid_2d tiny_deep_8_bfloat16 4 4 \
    tests/data "$@" -w 1 -r 2 --backend xgmi -d 0,0,0,0 --compute sleep --no-topology > gpurun_out/il_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/il_steps.log
  return $rc
}
step 1f1b --pp-schedule 1f1b && step il_v1 --pp-schedule interleaved --pp-virtual 1 && \
  step il_v2 --pp-schedule interleaved --pp-virtual 2 && step il_v3 --pp-schedule interleaved --pp-virtual 3
