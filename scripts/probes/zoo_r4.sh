#!/bin/bash
# Round 4: GEMM numerics after the tile-order change, then the model-zoo FFN shapes with the default dispatch
# (bf16 + fp8, interleaved vs torch) - the round-3 table's shapes (model_zoo_gemm.sh).
set -o pipefail
mkdir -p gpurun_out/zoo4
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/zoo4/pytest.log 2>&1 || exit $?
bash scripts/probes/model_zoo_gemm.sh || exit $?
cp gpurun_out/zoo/*.txt gpurun_out/zoo4/
