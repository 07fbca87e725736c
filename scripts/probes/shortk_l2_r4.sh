#!/bin/bash
# Round 4: L2 behaviour of the fp8 short-K GEMM (8192 x 4096 x 1024) vs the vendor: hits, misses, HBM read
# requests (one TCC pass: HIT, MISS, EA0_RDREQ + GRBM) and write requests (second pass), over gemm_bench.
set -o pipefail
O=gpurun_out/shortk_l2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p1 -o g -- \
  python3 -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 5 --shapes 8192x4096x1024,8192x8192x1024 --rounds 2 --iters 10 \
  > $O/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_RDREQ_DRAM_sum GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o g -- \
  python3 -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 5 --shapes 8192x4096x1024,8192x8192x1024 --rounds 2 --iters 10 \
  > $O/p2.log 2>&1 || exit $?
echo done > $O/done.txt
