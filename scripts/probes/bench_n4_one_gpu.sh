#!/bin/bash
# The N = 8 bench.py path (exactness pass, headline, C5, link_bench, C3 / C4
# hybrids + C4 --ep-overlap, xgmi secondaries) as 4 torchrun ranks sharing
# GPU 0 over the xgmi kernels, tiny models, the hybrids forced on with
# 4-rank shapes. 4, not 8: every rank's child-process blocks also open the
# GPU and the box allows 16 processes on it. Mechanics only: RCCL refuses
# several ranks on one device, so its blocks are the driver's 8-GPU run's.
set -u
mkdir -p gpurun_out/bench_n4
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=60
D=tests/data
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=4 --master-addr 127.0.0.1 \
  --master-port 29555 bench.py --gpus 4 --steps 2 --warmup 1 --backend xgmi --devices 0,0,0,0 \
  --model tiny_dense_8_bfloat16 --base-path $D --units 4 --c5-model tiny_dense_8_bfloat16 --c5-steps 3 \
  --exact-sizes 4097,300000 --link-sizes 1048576 --hybrids on --c3-model tiny_deep_8_bfloat16 --c3 2,4,2 \
  --c4-model tiny_moe_8_bfloat16 --c4 2,8,2 > gpurun_out/bench_n4/line.json 2> gpurun_out/bench_n4/err.log
