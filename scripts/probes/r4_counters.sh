#!/bin/bash
# Round 4 GPU pass 2: the fixed graph-mode mutation tests, the headline's
# timeline with deadline-bounded compute spans, and the rocprof counters of the
# headline with device gates (MFMA busy on the deadline grid must hold).
set -u
O=gpurun_out/r4c
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
step pytest 300 python -u -m pytest tests/test_commtest.py -v -m gpu -k "injected or exactness" \
  -p no:cacheprovider --timeout 120 --timeout-method thread
F="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 1 -r 2 --quiet --silent"
step tl_on 150 env DLNB_NO_TORCH=1 $F --timeline $O/tl_on.json --json $O/tl_on_report.json
step tl_on_sum 60 python -m dlnetbench_amd timeline $O/tl_on.json --check
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="bench.py --c5-model none --stretch-steps 0"
step cnt_trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/cnt_trace -o bench -- python3 $B --steps 2 --warmup 1 --json $O/bench_cnt_report.json
step cnt_pmc_a 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 FETCH_SIZE --output-format csv -d $O/cnt_pmc_a -o a -- python3 $B --steps 1 --warmup 0 --no-graph
step cnt_pmc_b 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d $O/cnt_pmc_b -o b -- python3 $B --steps 1 --warmup 0 --no-graph
step cnt_merge 60 python -m dlnetbench_amd.tools.prof_merge $O/bench_cnt_report.json $O/cnt_trace $O/cnt_pmc_a $O/cnt_pmc_b -o $O/bench_counters.json
echo done >> $O/steps.log
