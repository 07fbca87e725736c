#!/bin/bash
# Round 4: the model-zoo FFN shapes (model_zoo_gemm.sh) with the default dispatch (narrow tiles where they save
# rounds, else square) under tile-order groups 8 and 4 (DLNB_GEMM_GROUP), bf16 and fp8, interleaved vs torch.
set -o pipefail
mkdir -p gpurun_out/zoog
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=8192x768x3072,8192x1024x4096,8192x1280x5120,8192x1792x6400,8192x3072x768,8192x4096x1024,8192x4096x14336,8192x5120x1280,8192x6400x1792,8192x8192x28672,8192x14336x4096,8192x28672x8192
for d in fp8 bf16; do
  timeout -k 10 500 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --ab DLNB_GEMM_GROUP=8,4 --rounds 5 \
    --shapes $S > gpurun_out/zoog/$d.txt 2>&1 || exit $?
done
echo done > gpurun_out/zoog/done.txt
