# Square MX fp8 kernel with the explicit start-of-K-tile lgkmcnt (LDS WAR ordering): numerics + TF/s vs _scaled_mm.
set -o pipefail
mkdir -p gpurun_out/war
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/war/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/war/pytest.log; exit 1; }
tail -2 gpurun_out/war/pytest.log
timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 0 --rounds 7 --shapes 4096x4096x4096,8192x8192x8192,8192x14336x4096,8192x1280x5120 > gpurun_out/war/fp8.txt 2>&1
grep -h '^{' gpurun_out/war/fp8.txt
