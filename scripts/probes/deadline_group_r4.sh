#!/bin/bash
# Round 4: tile-order group of the headline's bf16 deadline GEMM (8-phase per-tile kernel; DLNB_DEADLINE_GROUP 8 vs
# 4): MFMA work per clock inside the headline step (one eager step under PMC + a kernel trace each, prof_merge).
set -u
O=gpurun_out/dgroup
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="bench.py --c5-model none --stretch-steps 0"
for g in 8 4 8 4; do
  T=$O/g${g}_$RANDOM
  mkdir -p $T
  env DLNB_DEADLINE_GROUP=$g timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $T/trace -o bench -- python3 $B --steps 2 --warmup 1 --json $T/report.json > $T/trace.log 2>&1 || exit 1
  env DLNB_DEADLINE_GROUP=$g timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv -d $T/pmc -o a -- python3 $B --steps 1 --warmup 0 --no-graph > $T/pmc.log 2>&1 || exit 1
  timeout -k 10 60 python -m dlnetbench_amd.tools.prof_merge $T/report.json $T/trace $T/pmc -o $T/counters.json > $T/merge.log 2>&1 || exit 1
  echo "g=$g $T ok" >> $O/steps.log
done
