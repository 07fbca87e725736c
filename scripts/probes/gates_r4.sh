#!/bin/bash
# Round 4: device gates + chained deadlines in the FSDP headline (N = 1).
#   1. the gate / chain kernel tests
#   2. bench.py headline, gates on (default) and off (DLNB_DEVICE_GATES=0), interleaved
#   3. --timeline of the headline config with gates on and off, summarised
# Each GPU step under its own timeout, chained with && (stop at the first failure).
set -u
O=gpurun_out/gates
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
B="python bench.py --steps 5 --warmup 2 --c5-model none --stretch-steps 0"
timeout -k 10 180 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "chain or gate or deadline" \
  -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 &&
timeout -k 10 200 $B --json $O/bench_on_report.json > $O/bench_on.json 2> $O/bench_on.log &&
DLNB_DEVICE_GATES=0 timeout -k 10 200 $B > $O/bench_off.json 2> $O/bench_off.log &&
timeout -k 10 200 $B > $O/bench_on2.json 2> $O/bench_on2.log &&
DLNB_NO_TORCH=1 timeout -k 10 150 build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph \
  -w 1 -r 2 --quiet --silent --timeline $O/tl_on.json --json $O/tl_on_report.json > $O/tl_on.log 2>&1 &&
python -m dlnetbench_amd timeline $O/tl_on.json --check > $O/tl_on_summary.txt 2>&1 &&
DLNB_NO_TORCH=1 DLNB_DEVICE_GATES=0 timeout -k 10 150 build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl \
  --compute gemm --graph -w 1 -r 2 --quiet --silent --timeline $O/tl_off.json > $O/tl_off.log 2>&1 &&
python -m dlnetbench_amd timeline $O/tl_off.json --check > $O/tl_off_summary.txt 2>&1
echo "rc=$?" >> $O/done.txt
