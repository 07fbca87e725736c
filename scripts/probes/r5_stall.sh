#!/bin/bash
# Round 5, VERDICT r4 #5: the slow replay every 16th under the single graph (DLNB_LANE_GRAPHS=0) against the HIP
# runtime's batch / signal-pool knobs, the lane graphs for comparison, and a kernel trace of the single graph.
set -u
O=${O:-gpurun_out/r5_stall}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { echo "$1 start $(date +%s)" >> $O/steps.log; }
ok() { echo "$1 ok" >> $O/steps.log; }
run() {  # name env... -- command
  local n=$1; shift
  step $n
  env "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?" >> $O/steps.log; exit 1; }
  ok $n
}
H="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 4 -r 64 --time-scale 0.05 --quiet --silent"
run s_base DLNB_LANE_GRAPHS=0 timeout -k 10 150 $H --json $O/s_base.json
run l_base timeout -k 10 150 $H --json $O/l_base.json
if [ "${KNOBS:-1}" = 1 ]; then
run s_active DLNB_LANE_GRAPHS=0 ROC_ACTIVE_WAIT_TIMEOUT=1000000 timeout -k 10 150 $H --json $O/s_active.json
run s_cpuwait DLNB_LANE_GRAPHS=0 ROC_CPU_WAIT_FOR_SIGNAL=0 timeout -k 10 150 $H --json $O/s_cpuwait.json
run s_batch DLNB_LANE_GRAPHS=0 DEBUG_CLR_MAX_BATCH_SIZE=4096 timeout -k 10 150 $H --json $O/s_batch.json
run s_sigpool DLNB_LANE_GRAPHS=0 ROC_SIGNAL_POOL_SIZE=1024 timeout -k 10 150 $H --json $O/s_sigpool.json
fi
unset DLNB_NO_TORCH
if [ "${BENCH:-0}" = 1 ]; then
  step bench
  timeout -k 10 900 python bench.py --steps 20 --warmup 5 --json $O/bench_report.json > $O/bench.json 2> $O/bench.err || { echo "bench rc=$?" >> $O/steps.log; exit 1; }
  ok bench
fi
