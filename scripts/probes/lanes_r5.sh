#!/bin/bash
# Round 5: lane graphs (one linear graph per stream, gates instead of edges) on the C5 step and a time-scaled
# headline FSDP, against the single graph (DLNB_LANE_GRAPHS=0) and eager; the lane probe; a kernel trace of C5
# with lanes for the queue ids.
set -u
O=gpurun_out/lanes
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5
step() { echo "$1 start $(date +%s)" >> $O/steps.log; }
ok() { echo "$1 ok" >> $O/steps.log; }
step probe
timeout -k 10 60 build/bin/lane_probe > $O/probe.txt 2>&1 || { echo "probe rc=$?" >> $O/steps.log; exit 1; }
ok probe
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm -w 5 -r 30 --quiet --silent"
step c5_lanes
timeout -k 10 120 $C5 --graph --json $O/c5_lanes.json > $O/c5_lanes.log 2>&1 || { echo "c5_lanes rc=$?" >> $O/steps.log; exit 1; }
ok c5_lanes
step c5_single
DLNB_LANE_GRAPHS=0 timeout -k 10 120 $C5 --graph --json $O/c5_single.json > $O/c5_single.log 2>&1 || { echo "c5_single rc=$?" >> $O/steps.log; exit 1; }
ok c5_single
step c5_eager
timeout -k 10 120 $C5 --json $O/c5_eager.json > $O/c5_eager.log 2>&1 || { echo "c5_eager rc=$?" >> $O/steps.log; exit 1; }
ok c5_eager
step c5_geo
timeout -k 10 120 $C5 --graph --dp-bucket-ratio 0.7 --json $O/c5_geo_lanes.json > $O/c5_geo.log 2>&1 || { echo "c5_geo rc=$?" >> $O/steps.log; exit 1; }
ok c5_geo
H="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 2 -r 10 --time-scale 0.05 --quiet --silent"
step head_lanes
timeout -k 10 150 $H --json $O/head_lanes.json > $O/head_lanes.log 2>&1 || { echo "head_lanes rc=$?" >> $O/steps.log; exit 1; }
ok head_lanes
step head_single
DLNB_LANE_GRAPHS=0 timeout -k 10 150 $H --json $O/head_single.json > $O/head_single.log 2>&1 || { echo "head_single rc=$?" >> $O/steps.log; exit 1; }
ok head_single
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step trace
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o c5 -- \
  build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 2 -r 4 --quiet --silent \
  > $O/trace.log 2>&1 || { echo "trace rc=$?" >> $O/steps.log; exit 1; }
ok trace
# the slow replay every 16 timed iterations - HIP API + kernel trace of a 40-replay headline
step trace16
timeout -k 10 240 rocprofv3 --hip-trace --kernel-trace --output-format csv -d $O/trace16 -o head -- \
  build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 1 -r 40 --time-scale 0.05 \
  --quiet --silent --json $O/trace16.json > $O/trace16.log 2>&1 || { echo "trace16 rc=$?" >> $O/steps.log; exit 1; }
ok trace16
echo done >> $O/steps.log
