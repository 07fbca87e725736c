#!/bin/bash
# Round 4 verification pass: the GPU test suite, the driver's N = 1 bench, and the N > 1 bench path as 4 ranks
# sharing the GPU over the xgmi kernels (wall budget, exactness pass with the new patterns, every block).
set -u
bash scripts/gpu_check.sh pytest benchdriver || exit $?
grep -q "fatal" gpurun_out/steps.log && exit 3
bash scripts/probes/bench_n4_one_gpu.sh
echo "bench_n4 rc=$?" >> gpurun_out/steps.log
