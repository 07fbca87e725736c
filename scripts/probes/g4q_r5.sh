#!/bin/bash
# Round 5: the one-wave-per-SIMD square kernel on the quarter schedule (ktile_q, DLNB_G4_SCHED=q): numerics
# (K-tile counts, deadline tiles), then one-shot throughput against the streaming / per-tile half schedule,
# the 8-phase default and hipBLASLt (interleaved rounds, one process).
# (The kernel and test changes it ran against: profiles/gemm_r5/quarter_schedule.diff.txt; not kept.)
set -u
O=gpurun_out/g4q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $O/steps.log
  timeout -k 10 "$to" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >> $O/steps.log
  case $rc in 0) return 0 ;; *) echo "fatal rc=$rc in $name" >> $O/steps.log; exit $rc ;; esac
}
step pytest 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "k_tile_counts or deadline_gemm_numerics" \
  -p no:cacheprovider --timeout 120 --timeout-method thread
step gemm 400 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16 --variants 0,5 --rounds 5 --ab DLNB_G4_SCHED=s,t,q \
  --shapes 8192x4096x14336,8192x14336x4096,8192x8192x8192,4096x4096x4096
echo done >> $O/steps.log
