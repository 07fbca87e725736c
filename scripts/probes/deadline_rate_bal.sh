#!/bin/bash
# bf16 deadline GEMM: plain 8-phase (DLNB_GEMM_BF16_DL_BAL=0) vs balanced reads (1); PMC TF/s over 5 x 20 ms.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for e in 0 1; do
  DLNB_GEMM_BF16_DL_BAL=$e timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d gpurun_out/dbal$e -o drate -- python3 scripts/probes/deadline_rate.py \
    > gpurun_out/dbal$e.log 2>&1 || exit $?
  python3 scripts/probes/pmc_table.py gpurun_out/dbal$e >> gpurun_out/dbal_table.txt
done
