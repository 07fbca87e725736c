#!/bin/bash
# Two PMC passes over GEMM variants (VARIANTS, default "2,3"; "t" = torch/hipBLASLt;
# DTYPE bf16|fp8, SHAPE MxNxK, default 8192^3), then a per-kernel table (scripts/probes/pmc_table.py).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
V=${VARIANTS:-2,3}
DT=${DTYPE:-bf16}
SH=${SHAPE:-8192x8192x8192}
MOPS=SQ_INSTS_VALU_MFMA_MOPS_BF16
[ "$DT" = fp8 ] && MOPS=SQ_INSTS_VALU_MFMA_MOPS_F8
timeout -s KILL 90 rocprofv3 --pmc $MOPS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/gpmc1 -o g \
  -- python3 scripts/probes/gemm_pmc.py "$V" "$DT" "$SH" > gpurun_out/gpmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
  SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/gpmc2 -o g \
  -- python3 scripts/probes/gemm_pmc.py "$V" "$DT" "$SH" > gpurun_out/gpmc2.log 2>&1 || exit $?
python3 scripts/probes/pmc_table.py gpurun_out/gpmc1 gpurun_out/gpmc2 > gpurun_out/gpmc_table.txt
