# Narrow-tile one-shot GEMM (gemm_4wave_fp8.hip, gemm_4wave_narrow_kernel): numerics, then
# TF/s vs torch (hipBLASLt) with the narrow tiles (default) and pinned to the square tile
# (DLNB_GEMM_NARROW_NF=8), bf16 and fp8. Output: gpurun_out/nf/.
set -o pipefail
mkdir -p gpurun_out/nf
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "gemm" -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/nf/pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/nf/pytest.log; exit 1; }
tail -3 gpurun_out/nf/pytest.log
S8=8192x1280x5120,8192x1024x1280,8192x1536x6144,8192x768x3072,4096x4096x4096
SB=8192x1280x5120,8192x1024x4096,8192x1536x6144,8192x768x3072,8192x4096x14336
for d in fp8 bf16; do
  S=$([ $d = fp8 ] && echo $S8 || echo $SB)
  timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --rounds 5 --shapes $S > gpurun_out/nf/bench_${d}_nf.txt 2>&1
  DLNB_GEMM_NARROW_NF=8 timeout -k 10 300 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --rounds 5 --shapes $S > gpurun_out/nf/bench_${d}_sq.txt 2>&1
done
grep -h '^{' gpurun_out/nf/bench_*.txt
