#!/bin/bash
# Round 4: DP comm gates (each backward bucket raises a device gate, the comm lane waits for it on the device: no
# cross-stream graph edge, so the executor keeps each chain on one hardware queue) vs event waits, on the C5 step,
# graph and eager, with kernel traces of the graph runs (queue ids). Then the DP GPU tests.
set -u
O=gpurun_out/dpg
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm -w 5 -r 30 --quiet --silent"
for v in gates events gates_eager events_eager gates2; do
  case $v in gates|gates2) e="DLNB_DP_COMM_GATES=1"; g="--graph" ;; events) e="DLNB_DP_COMM_GATES=0"; g="--graph" ;;
    gates_eager) e="DLNB_DP_COMM_GATES=1"; g="" ;; events_eager) e="DLNB_DP_COMM_GATES=0"; g="" ;; esac
  env $e timeout -k 10 120 $C5 $g --json $O/c5_$v.json > $O/c5_$v.log 2>&1 || { echo "rc=$? $v" >> $O/steps.log; exit 1; }
  echo "$v ok" >> $O/steps.log
done
C5G="$C5 --dp-bucket-ratio 0.7 --graph"
env DLNB_DP_COMM_GATES=1 timeout -k 10 120 $C5G --json $O/c5_geo_gates.json > $O/c5_geo_gates.log 2>&1 || exit 1
env DLNB_DP_COMM_GATES=0 timeout -k 10 120 $C5G --json $O/c5_geo_events.json > $O/c5_geo_events.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for v in gates events; do
  if [ $v = gates ]; then e=1; else e=0; fi
  DLNB_DP_COMM_GATES=$e timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$v -o c5 -- $C5 --graph \
    > $O/trace_$v.log 2>&1 || { echo "trace rc=$? $v" >> $O/steps.log; exit 1; }
done
unset DLNB_NO_TORCH
timeout -k 10 300 python -u -m pytest tests/test_gpu_strategies.py -x -v -k "dp_" -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1
echo "pytest rc=$?" >> $O/steps.log
