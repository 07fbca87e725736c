#!/bin/bash
# Round 4, end of session: the GPU test suite and the driver's N = 1 bench on the final tree, then the N > 1
# paths on one GPU (4 ranks over xgmi; 2 ranks with the default backend -> RCCL refuses -> xgmi fallback).
set -u
bash scripts/gpu_check.sh pytest benchdriver || exit $?
grep -q "fatal" gpurun_out/steps.log && exit 3
bash scripts/probes/bench_n4_one_gpu.sh || exit $?
bash scripts/probes/fallback_two_ranks_one_gpu.sh
