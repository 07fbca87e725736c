#!/bin/bash
# Round 5: the lane-graph iteration end - compute program join + trailing pad node vs no pad vs the single graph,
# C5 and the time-scaled headline, a C5 kernel trace; optional bench.py headline A/B (BENCH=1).
set -u
O=${O:-gpurun_out/lanes_f}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { echo "$1 start $(date +%s)" >> $O/steps.log; }
ok() { echo "$1 ok" >> $O/steps.log; }
run() {  # name env... -- command
  local n=$1; shift
  step $n
  env "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?" >> $O/steps.log; exit 1; }
  ok $n
}
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm -w 5 -r 30 --quiet --silent --graph"
H="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 2 -r 10 --time-scale 0.05 --quiet --silent"
run c5_pad timeout -k 10 120 $C5 --json $O/c5_pad.json
run c5_nopad DLNB_LANE_TAIL_PAD=0 timeout -k 10 120 $C5 --json $O/c5_nopad.json
run c5_normprio DLNB_HIGH_PRIORITY_STREAMS=0 timeout -k 10 120 $C5 --json $O/c5_normprio.json
run head_normprio DLNB_HIGH_PRIORITY_STREAMS=0 timeout -k 10 150 $H --json $O/head_normprio.json
run trace_normprio DLNB_HIGH_PRIORITY_STREAMS=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_normprio -o c5 -- \
  build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 2 -r 4 --quiet --silent
run c5_nojoin DLNB_COMPUTE_PROGRAMS=0 timeout -k 10 120 $C5 --json $O/c5_nojoin.json
run c5_single DLNB_LANE_GRAPHS=0 timeout -k 10 120 $C5 --json $O/c5_single.json
run head_pad timeout -k 10 150 $H --json $O/head_pad.json
run head_single DLNB_LANE_GRAPHS=0 timeout -k 10 150 $H --json $O/head_single.json
run trace timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o c5 -- \
  build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 2 -r 4 --quiet --silent
run trace_single DLNB_LANE_GRAPHS=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_single -o c5 -- \
  build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 2 -r 4 --quiet --silent
unset DLNB_NO_TORCH DLNB_GATE_TIMEOUT_S
if [ "${BENCH:-0}" = 1 ]; then
  step bench_lanes
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0 > $O/bench_lanes.json 2> $O/bench_lanes.err || { echo "bench rc=$?" >> $O/steps.log; exit 1; }
  ok bench_lanes
  step bench_single
  DLNB_LANE_GRAPHS=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0 > $O/bench_single.json 2> $O/bench_single.err || { echo "bench rc=$?" >> $O/steps.log; exit 1; }
  ok bench_single
fi
echo done >> $O/steps.log
