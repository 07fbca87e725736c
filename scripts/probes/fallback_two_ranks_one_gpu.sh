#!/bin/bash
# Round 4: bench.py's N > 1 fallback on real hardware. Two torchrun ranks share GPU 0 with the default backend
# (auto = RCCL): RCCL refuses two ranks on one device, so the exactness pass fails RCCL and proves the xgmi
# kernels, the headline runs as a bounded child on RCCL, fails, and is timed again on xgmi; the line must carry a
# value with headline_fallback. Tiny models; the RCCL-only blocks fail fast and are reported.
set -u
O=gpurun_out/fb2
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=60
D=tests/data
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
  --master-port 29557 bench.py --gpus 2 --steps 2 --warmup 1 --devices 0,0 --wall-budget-s 300 \
  --model tiny_dense_8_bfloat16 --base-path $D --units 4 --c5-model tiny_dense_8_bfloat16 --c5-steps 3 \
  --exact-sizes 4097,300000 --link-sizes 1048576 > $O/line.json 2> $O/err.log
echo "rc=$?" >> $O/steps.log
