#!/bin/bash
# PMC of the fp8 deadline GEMM: 2-phase (DLNB_GEMM_8PHASE=0) vs 8-phase schedule.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
for e in 0 1; do
  DLNB_GEMM_8PHASE=$e timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d gpurun_out/frate$e -o drate -- python3 scripts/probes/deadline_rate.py fp8 \
    > gpurun_out/frate$e.log 2>&1 || exit $?
done
