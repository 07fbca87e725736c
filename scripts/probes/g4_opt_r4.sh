#!/bin/bash
# Round 4: schedule options of the one-wave-per-SIMD square GEMMs (gemm_4wave_fp8.hip OPT / DLNB_G4_OPT):
# OPT_MAIN (clamp-free main K-loop staging, compile-time buffer parity: fewer SALU per MFMA) and OPT_ROWS
# (bf16: a row's lo K-steps then its hi ones, no s_nop between same-accumulator MFMAs). Numerics first,
# then one-shot TF/s interleaved against torch, fp8 and bf16. (After this A/B the main loop became
# unconditional and the row order was dropped; DLNB_G4_OPT no longer exists: profiles/gemm_g4_main_r4.md.)
set -u
O=gpurun_out/g4opt
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
step pytest 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "4wave_schedule or deadline_gemm_numerics" \
  -p no:cacheprovider --timeout 120 --timeout-method thread
S=8192x4096x14336,8192x14336x4096,8192x8192x8192,4096x4096x4096,8192x4096x1024
step fp8 300 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 5 --ab DLNB_G4_OPT=0,1 --rounds 5 --shapes $S
step bf16 400 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16 --variants 5 --ab DLNB_G4_OPT=0,1,2,3 --rounds 5 \
  --shapes 8192x4096x14336,8192x14336x4096,8192x8192x8192,4096x4096x4096
step bf16_8p 300 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16 --variants 0 --rounds 5 \
  --shapes 8192x4096x14336,8192x14336x4096,8192x8192x8192,4096x4096x4096
echo done >> $O/steps.log
