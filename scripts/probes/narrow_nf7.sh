# nf = 7 narrow tiles (256 x 224): GEMM numerics, then the GPT-2-XL stand-in shapes (N = 1792) with the default
# (nf = 7) and pinned square tiles, bf16 and fp8. Output: gpurun_out/nf7/.
set -o pipefail
mkdir -p gpurun_out/nf7
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/nf7/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/nf7/pytest.log; exit 1; }
tail -2 gpurun_out/nf7/pytest.log
S=8192x1792x6400,8192x1792x1792
for d in bf16 fp8; do
  timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --rounds 5 --shapes $S > gpurun_out/nf7/${d}_nf.txt 2>&1
  DLNB_GEMM_NARROW_NF=8 timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --rounds 5 --shapes $S > gpurun_out/nf7/${d}_sq.txt 2>&1
done
grep -H '^{' gpurun_out/nf7/*.txt
