#!/bin/bash
# xgmi kernel throughput sweep on one MI355X: W ranks sharing GPU 0 (IPC within
# the device: local HBM through the windows, not xGMI links), window memory
# type x block cap, HIP-graph replayed ops (launch overhead out of the way),
# plus the local D2D copy roofline. Each memory type is first checked exactly
# (the bench only runs if it passes). Output: gpurun_out/xgmi_sweep.jsonl
# usage: scripts/xgmi_sweep.sh [W] [mem types] [block caps] [sizes]
# EXTRA="--registered" runs the zero-copy paths (registered peer buffers).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=20
W=${1:-2}
MEMS=${2:-"uncached fine coarse"}
BLOCKS=${3:-"64 128 256 512 1024"}
SIZES=${4:-"1048576,16777216,67108864,268435456"}
DEVS=$(python3 -c "print(','.join(['0']*$W))")
OUT=gpurun_out/xgmi_sweep.jsonl
run() {  # label timeout args...
  local label=$1 to=$2; shift 2
  timeout -k 10 "$to" python -m dlnetbench_amd.utils.launch -n "$W" --timeout $((to - 20)) build/bin/dlnb commtest \
    --backend xgmi -d "$DEVS" "$@" > gpurun_out/sweep_cur.log 2> gpurun_out/sweep_cur.err
  local rc=$?
  grep '^{' gpurun_out/sweep_cur.log | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); d.update($label); print(json.dumps(d))" >> $OUT
  echo "$label rc=$rc" >> gpurun_out/xgmi_sweep_steps.log
  case $rc in 0|3) return 0 ;; *) tail -20 gpurun_out/sweep_cur.err >> gpurun_out/xgmi_sweep_steps.log; exit $rc ;; esac
}
for mem in $MEMS; do
  export DLNB_XGMI_MEM=$mem
  DLNB_XGMI_REGION_MB=1 DLNB_XGMI_P2P_MB=1 run "{'mem':'$mem','W':$W,'check':'eager'}" 120 --sizes 1,100,4097,300000,1048583 ${EXTRA:-}
  run "{'mem':'$mem','W':$W,'check':'graph'}" 120 --graph --sizes 1,4097,1048583 ${EXTRA:-}
  if ! tail -2 $OUT | grep -q '"ok": true'; then echo "$mem: check failed, no bench" >> gpurun_out/xgmi_sweep_steps.log; continue; fi
  for b in $BLOCKS; do
    DLNB_XGMI_BLOCKS=$b run "{'mem':'$mem','W':$W,'blocks':$b,'extra':'${EXTRA:-}'}" 200 --bench --graph --iters 10 --warmup 3 --sizes $SIZES ${EXTRA:-}
  done
done
