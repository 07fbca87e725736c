#!/bin/bash
# PMC of the bf16 deadline GEMM vs the one-shot kernel at the headline shape:
# MFMA busy / MOPS per clock, wave time waiting (any, LDS), one pass each.
set -u
out=gpurun_out/deadline_pmc
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in ${MODES:-oneshot deadline}; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_${MOPS:-BF16} SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS \
    SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $out/$m -o p -- \
    python3 scripts/probes/deadline_vs_oneshot.py $m ${SHAPE:-} > $out/$m.log 2>&1 || exit 1
  timeout -k 5 60 python3 -m dlnetbench_amd.tools.prof_merge - $out/$m -o $out/$m.json > /dev/null || exit 1
done
