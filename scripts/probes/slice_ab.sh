#!/bin/bash
# A/B of the deadline GEMM's relaunch slice (DLNB_GEMM_SLICE_US, compute.cpp)
# on the headline FSDP step at N = 1: for each slice length, a short bench.py
# run (iteration time, comm_bound block) and one PMC pass of one eagerly
# enqueued iteration (MFMA busy / TF/s of the deadline kernel, merged by
# tools/prof_merge.py). VERDICT r2 "next round" item 5.
set -u
out=gpurun_out/slice_ab
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for s in ${SLICES:-500 5000 1000000}; do
  timeout -k 10 240 env DLNB_GEMM_SLICE_US=$s python3 bench.py --steps 3 --warmup 1 --stretch-steps 0 \
    --no-c5-ctas-ab --c5-bucket-ratio 0 --json $out/report_$s.json > $out/bench_$s.json 2> $out/bench_$s.err || exit 1
  timeout -k 10 240 env DLNB_GEMM_SLICE_US=$s rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv -d $out/pmc_$s -o p -- \
    python3 bench.py --c5-model none --stretch-steps 0 --steps 1 --warmup 0 --no-graph > $out/pmc_$s.log 2>&1 || exit 1
  timeout -k 10 60 python3 -m dlnetbench_amd.tools.prof_merge - $out/pmc_$s -o $out/counters_$s.json > /dev/null || exit 1
done
