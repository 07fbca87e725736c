#!/bin/bash
# Round 5: per-lane linear graphs joined by device gates (scripts/probes/src/lane_probe.hip): queue independence of
# the streams a rank uses, concurrent capture of two streams, replay timing; then a kernel trace for queue ids.
set -u
O=gpurun_out/lane
mkdir -p $O
timeout -k 10 60 build/bin/lane_probe > $O/probe.txt 2>&1 || { echo "probe rc=$?" >> $O/steps.log; exit 1; }
GPU_MAX_HW_QUEUES=2 timeout -k 10 60 build/bin/lane_probe > $O/probe_q2.txt 2>&1 || { echo "probe q2 rc=$?" >> $O/steps.log; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o lane -- build/bin/lane_probe \
  > $O/trace.log 2>&1 || { echo "trace rc=$?" >> $O/steps.log; exit 1; }
echo done >> $O/steps.log
