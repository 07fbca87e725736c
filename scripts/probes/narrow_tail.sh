# Narrow tiles for a partial last round of square tiles (gemm_narrow_nf): numerics, then TF/s with the
# default choice and with DLNB_GEMM_NARROW_NF=8 (square), bf16 and fp8. Output: gpurun_out/tail/.
set -o pipefail
mkdir -p gpurun_out/tail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/tail/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/tail/pytest.log; exit 1; }
tail -2 gpurun_out/tail/pytest.log
S=8192x5120x4096,8192x3072x4096,8192x2560x8192,8192x5120x5120
for d in bf16 fp8; do
  timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --rounds 5 --shapes $S > gpurun_out/tail/${d}_nf.txt 2>&1
  DLNB_GEMM_NARROW_NF=8 timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --rounds 5 --shapes $S > gpurun_out/tail/${d}_sq.txt 2>&1
done
grep -H '^{' gpurun_out/tail/*.txt
