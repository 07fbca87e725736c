#!/bin/bash
# Round 4: what the host's per-iteration timing adds to the headline's device span at N = 1.
#   1. timeline of the headline config with DLNB_TIMELINE_EDGES stamps around each graph launch
#   2. bench.py, interleaved: default (pre-armed graph loop + measured clock rate),
#      DLNB_CLOCK_CAL_MS=0 (nominal 100 MHz ticks), DLNB_PREARM=0 DLNB_CLOCK_CAL_MS=0 (round-4 loop)
set -u
O=gpurun_out/hostb
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
F="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 1 -r 4 --quiet --silent"
B="python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0"
DLNB_NO_TORCH=1 DLNB_TIMELINE_EDGES=1 timeout -k 10 150 $F --timeline $O/tle.json --json $O/tle_report.json > $O/tle.out 2>&1 &&
timeout -k 10 60 python -m dlnetbench_amd timeline $O/tle.json --check > $O/tle_sum.txt 2>&1 &&
timeout -k 10 240 $B > $O/bench_default.out 2> $O/bench_default.err &&
DLNB_CLOCK_CAL_MS=0 timeout -k 10 240 $B > $O/bench_nominal.out 2> $O/bench_nominal.err &&
DLNB_PREARM=0 DLNB_CLOCK_CAL_MS=0 timeout -k 10 240 $B > $O/bench_old.out 2> $O/bench_old.err &&
timeout -k 10 240 $B > $O/bench_default2.out 2> $O/bench_default2.err &&
echo done >> $O/steps.log
