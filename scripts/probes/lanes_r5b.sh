#!/bin/bash
# Round 5: lane graphs with compute programs (one persistent deadline kernel per lane iteration) on C5 and a
# time-scaled headline, against lanes without programs and the single graph; a C5 kernel trace; the lane / timer /
# deadline GPU tests.
set -u
O=${O:-gpurun_out/lanes_b}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1 DLNB_GATE_TIMEOUT_S=5
step() { echo "$1 start $(date +%s)" >> $O/steps.log; }
ok() { echo "$1 ok" >> $O/steps.log; }
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm -w 5 -r 30 --quiet --silent --graph"
step c5_prog
timeout -k 10 120 $C5 --json $O/c5_prog.json > $O/c5_prog.log 2>&1 || { echo "c5_prog rc=$?" >> $O/steps.log; exit 1; }
ok c5_prog
step c5_noprog
DLNB_COMPUTE_PROGRAMS=0 timeout -k 10 120 $C5 --json $O/c5_noprog.json > $O/c5_noprog.log 2>&1 || { echo "c5_noprog rc=$?" >> $O/steps.log; exit 1; }
ok c5_noprog
step c5_single
DLNB_LANE_GRAPHS=0 timeout -k 10 120 $C5 --json $O/c5_single.json > $O/c5_single.log 2>&1 || { echo "c5_single rc=$?" >> $O/steps.log; exit 1; }
ok c5_single
step c5_geo
timeout -k 10 120 $C5 --dp-bucket-ratio 0.7 --json $O/c5_geo.json > $O/c5_geo.log 2>&1 || { echo "c5_geo rc=$?" >> $O/steps.log; exit 1; }
ok c5_geo
H="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 2 -r 10 --time-scale 0.05 --quiet --silent"
step head_prog
timeout -k 10 150 $H --json $O/head_prog.json > $O/head_prog.log 2>&1 || { echo "head_prog rc=$?" >> $O/steps.log; exit 1; }
ok head_prog
step head_single
DLNB_LANE_GRAPHS=0 timeout -k 10 150 $H --json $O/head_single.json > $O/head_single.log 2>&1 || { echo "head_single rc=$?" >> $O/steps.log; exit 1; }
ok head_single
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step trace
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o c5 -- \
  build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm --graph -w 2 -r 4 --quiet --silent \
  > $O/trace.log 2>&1 || { echo "trace rc=$?" >> $O/steps.log; exit 1; }
ok trace
unset DLNB_NO_TORCH DLNB_GATE_TIMEOUT_S
if [ "${BENCH:-0}" = 1 ]; then
  for m in lanes single; do
    step bench_$m
    if [ $m = single ]; then e="DLNB_LANE_GRAPHS=0"; else e=""; fi
    env $e timeout -k 10 300 python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0 \
      > $O/bench_$m.json 2> $O/bench_$m.err || { echo "bench_$m rc=$?" >> $O/steps.log; exit 1; }
    ok bench_$m
  done
fi
step tests
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_kernels.py \
  tests/test_gpu_strategies.py -m gpu -k "deadline or graph_replay or exposed or prearm or comm_gates or chain" \
  > $O/tests.log 2>&1 || { echo "tests rc=$?" >> $O/steps.log; exit 1; }
ok tests
echo done >> $O/steps.log
