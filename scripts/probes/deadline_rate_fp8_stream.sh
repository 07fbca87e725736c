#!/bin/bash
# fp8 deadline GEMM on the one-wave-per-SIMD kernel: per-tile (DLNB_GEMM_FP8_DL_STREAM=0) vs streaming (1).
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
rm -f gpurun_out/fdst_table.txt
for e in 0 1; do
  DLNB_GEMM_FP8_DL_STREAM=$e timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F8 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
    --kernel-trace --output-format csv -d gpurun_out/fdst$e -o drate -- python3 scripts/probes/deadline_rate.py fp8 \
    > gpurun_out/fdst$e.log 2>&1 || exit $?
  echo "DL_STREAM=$e" >> gpurun_out/fdst_table.txt
  python3 scripts/probes/pmc_table.py gpurun_out/fdst$e >> gpurun_out/fdst_table.txt
done
