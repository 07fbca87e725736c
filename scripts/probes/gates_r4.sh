#!/bin/bash
# Round 4: device gates + chained deadlines in the FSDP headline (N = 1).
#   1. the gate / chain kernel tests
#   2. bench.py headline, gates on (default) and off (DLNB_DEVICE_GATES=0), interleaved
#   3. --timeline of the headline config with gates on and off, summarised
# Each GPU step under its own timeout; a test failure (rc 1) continues, any
# other failure (timeout, abort, fault) stops the script.
set -u
O=gpurun_out/gates
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $O/steps.log
  timeout -k 10 "$to" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >> $O/steps.log
  case $rc in 0|1) return 0 ;; *) echo "fatal rc=$rc in $name" >> $O/steps.log; exit $rc ;; esac
}
B="python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0"
step pytest 180 python -u -m pytest tests/test_gpu_kernels.py -v -k "chain or gate or deadline" \
  -p no:cacheprovider --timeout 120 --timeout-method thread
step bench_on 200 $B --json $O/bench_on_report.json
step bench_off 200 env DLNB_DEVICE_GATES=0 $B
step bench_on2 200 $B
export DLNB_NO_TORCH=1
F="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 1 -r 2 --quiet --silent"
step tl_on 150 $F --timeline $O/tl_on.json --json $O/tl_on_report.json
step tl_on_sum 60 python -m dlnetbench_amd timeline $O/tl_on.json --check
step tl_off 150 env DLNB_DEVICE_GATES=0 $F --timeline $O/tl_off.json
step tl_off_sum 60 python -m dlnetbench_amd timeline $O/tl_off.json --check
echo done >> $O/steps.log
