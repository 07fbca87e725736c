#!/bin/bash
# Round 5: K-stagger A/B on the one-wave-per-SIMD per-tile kernel (DLNB_G4_STAG="stride[:m|n|b]": block tiles
# start their K loop stride K-tiles apart by M-tile, N-tile or block, as the vendor kernel's StaggerU does).
# (The kernel change it ran against: profiles/gemm_r5/stagger.diff.txt; not kept.)
set -u
O=gpurun_out/g4stag
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
DLNB_G4_STAG=3 step pytest 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "k_tile_counts" \
  -p no:cacheprovider --timeout 120 --timeout-method thread
step gemm 500 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16 --variants 5 --rounds 5 \
  --ab DLNB_G4_STAG=0,1,2,8,2:n,2:b --shapes 8192x4096x14336,8192x14336x4096,8192x8192x8192,4096x4096x4096
echo done >> $O/steps.log
