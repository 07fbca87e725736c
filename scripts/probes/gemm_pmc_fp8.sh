#!/bin/bash
# PMC passes over the fp8 GEMMs at 8192^3: variant 8 (2-phase MX), variant 3 (8-phase MX) and torch._scaled_mm.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/fpmc1 -o g \
  -- python3 scripts/probes/gemm_pmc.py 8,3,t fp8 > gpurun_out/fpmc1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS \
  SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/fpmc2 -o g \
  -- python3 scripts/probes/gemm_pmc.py 8,3,t fp8 > gpurun_out/fpmc2.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/bpmc1 -o g \
  -- python3 scripts/probes/gemm_pmc.py 6,t bf16 > gpurun_out/bpmc1.log 2>&1
