#!/bin/bash
# Comm-bound ViT-H DP step (the bench's comm_bound block) on the captured HIP graph with the graph
# executor's queue count forced (DEBUG_HIP_FORCE_GRAPH_QUEUES; unset = HIP's default), and eager.
set -u
mkdir -p gpurun_out
A="vit_h_32_float8 8 . --no-topology -w 5 -r 50 --compute gemm --wire-dtype bf16 --json"
for q in default 1 2 4; do
  if [ $q = default ]; then env_q=""; else env_q="DEBUG_HIP_FORCE_GRAPH_QUEUES=$q"; fi
  env $env_q timeout -k 10 120 build/bin/dp $A gpurun_out/gq_$q.json --graph > gpurun_out/gq_$q.log 2>&1 || exit $?
  python3 -c "import json; d=json.load(open('gpurun_out/gq_$q.json'))['global']['dlnb']['iteration']; print('queues=$q', round(d['timed_ms_per_iter'],4), round(d['median_ms'],4))"
done
timeout -k 10 120 build/bin/dp $A gpurun_out/gq_eager.json > gpurun_out/gq_eager.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/gq_eager.json'))['global']['dlnb']['iteration']; print('eager', round(d['timed_ms_per_iter'],4), round(d['median_ms'],4))"
