# Paired 16-byte epilogue stores (csrc/kernels/store_pair.hpp): GEMM numerics, then one-shot TF/s vs torch
# (hipBLASLt / _scaled_mm) on the square shapes, where the epilogue of a one-tile-per-CU launch is exposed.
# Output: gpurun_out/epi/.
set -o pipefail
mkdir -p gpurun_out/epi
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/epi/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/epi/pytest.log; exit 1; }
tail -3 gpurun_out/epi/pytest.log
timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16 --variants 0 --rounds 5 --shapes 4096x4096x4096,8192x8192x8192,8192x4096x14336,8192x14336x4096 > gpurun_out/epi/bf16.txt 2>&1
timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 0 --rounds 5 --shapes 4096x4096x4096,8192x8192x8192,8192x14336x4096,8192x1280x5120 > gpurun_out/epi/fp8.txt 2>&1
grep -h '^{' gpurun_out/epi/*.txt
