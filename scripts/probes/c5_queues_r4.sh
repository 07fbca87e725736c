#!/bin/bash
# Round 4: the C5 step (graph) with the chained-deadline absorb cap, over the number of hardware queues the HIP
# graph executor spreads the replay over (DEBUG_HIP_FORCE_GRAPH_QUEUES; default = HIP's choice), with a kernel
# trace of the default to see which backward GEMM waits behind which all-reduce copy.
set -u
O=gpurun_out/c5q
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 5 -r 30 --quiet --silent"
for q in default 2 3 4 5 6 8 default; do
  if [ $q = default ]; then e=""; else e="DEBUG_HIP_FORCE_GRAPH_QUEUES=$q"; fi
  env $e timeout -k 10 120 $C5 --json $O/c5_q$q.json > $O/c5_q$q.log 2>&1 || { echo "rc=$? q=$q" >> $O/steps.log; exit 1; }
  echo "q=$q ok" >> $O/steps.log
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for q in 4 8; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_q$q -o c5 -- \
    $C5 > $O/trace_q$q.log 2>&1 || { echo "trace rc=$?" >> $O/steps.log; exit 1; }
done
echo done >> $O/steps.log
