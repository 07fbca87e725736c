#!/bin/bash
# Round 5: the lane-graph program rule (single graph when the compute lane is not one program), the clock
# reading's offset distribution (DLNB_CLOCK_DEBUG), and the periodic slow replay vs the HIP runtime's batch /
# signal-pool knobs: the time-scaled headline, 48 timed replays per variant.
set -u
O=${O:-gpurun_out/r5_fix}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step() { echo "$1 start $(date +%s)" >> $O/steps.log; }
ok() { echo "$1 ok" >> $O/steps.log; }
run() {  # name env... -- command
  local n=$1; shift
  step $n
  env "$@" > $O/$n.log 2>&1 || { echo "$n rc=$?" >> $O/steps.log; exit 1; }
  ok $n
}
export DLNB_NO_TORCH=1
H="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 4 -r 48 --time-scale 0.05 --quiet --silent"
run clock DLNB_CLOCK_DEBUG=1 timeout -k 10 120 build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 2 -r 4 --quiet --silent
run head_base timeout -k 10 150 $H --json $O/head_base.json
run head_single DLNB_LANE_GRAPHS=0 timeout -k 10 150 $H --json $O/head_single.json
run head_noprearm DLNB_PREARM=0 timeout -k 10 150 $H --json $O/head_noprearm.json
run head_base2 timeout -k 10 150 $H --json $O/head_base2.json
run head_noprearm2 DLNB_PREARM=0 timeout -k 10 150 $H --json $O/head_noprearm2.json
unset DLNB_NO_TORCH
if [ "${TESTS:-1}" = 1 ]; then
  run tests timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 170 --timeout-method thread \
    -k "graph_replay or prearm_and_clock or compute_stretch or program_lanes or exposed_comm or single_rank_secondaries"
fi
