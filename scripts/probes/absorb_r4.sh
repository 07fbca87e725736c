#!/bin/bash
# Round 4: the chained deadline's absorb cap (deadline_sync.hpp; DLNB_CHAIN_ABSORB_US, default 30 us). A replayed
# graph queued the C5 step's 5th backward GEMM behind the 4th bucket's all-reduce copy on one hardware queue
# (rocprof trace, c5_trace_r4.sh): ~85 us of wait the unbounded chain took out of that task's compute. With the
# cap, only launch hops are absorbed. A/B: cap 30 us vs effectively unbounded (1 s), headline and C5, graph and
# eager C5; then a kernel trace of the headline (every deadline task's dispatch length vs its table time).
set -u
O=gpurun_out/absorb
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> $O/steps.log
  timeout -k 10 "$to" "$@" > "$O/$name.out" 2> "$O/$name.err"
  local rc=$?
  echo "=== $name rc=$rc" >> $O/steps.log
  case $rc in 0) return 0 ;; *) echo "fatal rc=$rc in $name" >> $O/steps.log; exit $rc ;; esac
}
step pytest 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "deadline_chain or deadline_gate or deadline_gemm_numerics" \
  -p no:cacheprovider --timeout 120 --timeout-method thread
C5="build/bin/dp vit_h_32_float8 8 . --backend rccl --compute gemm -w 5 -r 20 --quiet --silent"
step c5_cap30 120 env DLNB_NO_TORCH=1 $C5 --graph --json $O/c5_cap30.json
step c5_capinf 120 env DLNB_NO_TORCH=1 DLNB_CHAIN_ABSORB_US=1000000 $C5 --graph --json $O/c5_capinf.json
step c5_eager 120 env DLNB_NO_TORCH=1 $C5 --json $O/c5_eager.json
step c5_cap30b 120 env DLNB_NO_TORCH=1 $C5 --graph --json $O/c5_cap30b.json
B="python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0"
step head_cap30 200 $B --json $O/head_cap30.json
step head_capinf 200 env DLNB_CHAIN_ABSORB_US=1000000 $B --json $O/head_capinf.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
step head_trace 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o head -- build/bin/fsdp llama3_8b_16_bfloat16 32 1 . \
  --backend rccl --compute gemm --graph -w 1 -r 2 --quiet --silent
echo done >> $O/steps.log
