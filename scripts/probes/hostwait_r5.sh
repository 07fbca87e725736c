#!/bin/bash
# Round 5: do the armed replay's host-memory polls slow the iteration's copies? host_wait polling tight for the
# whole wait (0) vs tight 50 us then one poll every ~4 us (DLNB_HOST_WAIT_TIGHT_US=50): one-rank hybrid_3d lanes
# (its 7-ms DP all-reduce copy), the FSDP headline and C5 at 0.05x / full.
set -u
O=${O:-gpurun_out/hostwait}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
H3="build/bin/hybrid_3d llama3_8b_16_bfloat16 1 4 1 . --backend rccl --compute gemm --graph --time-scale 0.05 --quiet --silent -w 3 -r 12"
HD="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph --time-scale 0.05 --quiet --silent -w 3 -r 12"
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph --quiet --silent -w 5 -r 30"
run1() {  # name env... -- cmd
  local n=$1; shift
  echo "$n start $(date +%s)" >> $O/steps.log
  env "$@" > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/steps.log; return $rc
}
for rep in a b; do
  run1 h3_t0_$rep DLNB_HOST_WAIT_TIGHT_US=0 timeout -k 10 120 $H3 --json $O/h3_t0_$rep.json || exit 1
  run1 h3_t50_$rep DLNB_HOST_WAIT_TIGHT_US=50 timeout -k 10 120 $H3 --json $O/h3_t50_$rep.json || exit 1
  run1 hd_t0_$rep DLNB_HOST_WAIT_TIGHT_US=0 timeout -k 10 120 $HD --json $O/hd_t0_$rep.json || exit 1
  run1 hd_t50_$rep DLNB_HOST_WAIT_TIGHT_US=50 timeout -k 10 120 $HD --json $O/hd_t50_$rep.json || exit 1
  run1 c5_t0_$rep DLNB_HOST_WAIT_TIGHT_US=0 timeout -k 10 120 $C5 --json $O/c5_t0_$rep.json || exit 1
  run1 c5_t50_$rep DLNB_HOST_WAIT_TIGHT_US=50 timeout -k 10 120 $C5 --json $O/c5_t50_$rep.json || exit 1
done
