#!/bin/bash
# Round 5: one-rank hybrid_3d (S=1, mb=4) lanes without a program: which part costs the 0.5-0.8 ms against the
# single graph (alternating stream sets, pre-arm, the tail pad), with a kernel trace of each.
set -u
O=${O:-gpurun_out/lanes_hyb_b}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
H="build/bin/hybrid_3d llama3_8b_16_bfloat16 1 4 1 . --backend rccl --compute gemm --graph --time-scale 0.05 --quiet --silent"
run1() {  # name env...
  local n=$1; shift
  echo "$n start $(date +%s)" >> $O/steps.log
  env "$@" timeout -k 10 120 $H -w 3 -r 12 --json $O/$n.json > $O/$n.log 2>&1
  local rc=$?; echo "$n rc=$rc" >> $O/steps.log; return $rc
}
run1 lanes X=1 && run1 single DLNB_LANE_GRAPHS=0 && run1 noalt DLNB_LANE_ALTERNATE=0 && run1 noprearm DLNB_PREARM=0 \
  && run1 nopad DLNB_LANE_TAIL_PAD=0 && run1 lanes_b X=1 && run1 single_b DLNB_LANE_GRAPHS=0 || exit 1
echo "trace start $(date +%s)" >> $O/steps.log
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_lanes -o h -- $H -w 2 -r 3 > $O/trace_lanes.log 2>&1 \
  && DLNB_LANE_GRAPHS=0 timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_single -o h -- $H -w 2 -r 3 > $O/trace_single.log 2>&1
echo "trace rc=$?" >> $O/steps.log
