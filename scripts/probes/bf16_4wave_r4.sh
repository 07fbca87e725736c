#!/bin/bash
# Round 4: the one-wave-per-SIMD square kernel with bf16 operands (variant 5 / DLNB_DEADLINE_BF16=4wave):
# numerics, one-shot throughput vs the 8-phase default and hipBLASLt, the headline with it as the deadline
# compute, and its PMC inside the headline (MFMA busy, clock).
set -u
O=gpurun_out/b4w
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $O/steps.log
  timeout -k 10 "$to" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >> $O/steps.log
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc in $name" >> $O/steps.log; exit $rc ;; esac
}
step pytest 240 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "bf16_matches or deadline_gemm_numerics" \
  -p no:cacheprovider --timeout 120 --timeout-method thread
step gemm 300 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16 --variants 0,5 --rounds 5 \
  --shapes 8192x4096x14336,8192x14336x4096,8192x8192x8192,4096x4096x4096,8192x8192x28672
B="python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0"
step bench_8p 200 $B
step bench_4w 200 env DLNB_DEADLINE_BF16=4wave $B
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="bench.py --c5-model none --stretch-steps 0 --steps 1 --warmup 0 --no-graph"
step pmc_4w 300 env DLNB_DEADLINE_BF16=4wave rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc_4w -o a -- python3 $P
step pmc_8p 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_LDS --kernel-trace --output-format csv -d $O/pmc_8p -o a -- python3 $P
echo done >> $O/steps.log
