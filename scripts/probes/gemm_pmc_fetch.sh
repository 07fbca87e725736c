#!/bin/bash
# HBM/L2 traffic of GEMM variants at 8192^3 (VARIANTS, default "6,5,t"):
# FETCH_SIZE / WRITE_SIZE (TCC) and the clock, then a per-kernel table.
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out
V=${VARIANTS:-6,5,t}
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 --kernel-trace --output-format csv \
  -d gpurun_out/gfetch1 -o g -- python3 scripts/probes/gemm_pmc.py "$V" > gpurun_out/gfetch1.log 2>&1 || exit $?
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --kernel-trace --output-format csv \
  -d gpurun_out/gfetch2 -o g -- python3 scripts/probes/gemm_pmc.py "$V" > gpurun_out/gfetch2.log 2>&1 || exit $?
python3 scripts/probes/pmc_table.py gpurun_out/gfetch1 gpurun_out/gfetch2 > gpurun_out/gfetch_table.txt
