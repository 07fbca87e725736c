# One-shot GEMM vs torch (hipBLASLt / _scaled_mm) on the FFN up / down projections of every model in models/*.json
# (M = 8192 tokens, N / K rounded up to 256), bf16 and fp8. Output: gpurun_out/zoo/.
set -o pipefail
mkdir -p gpurun_out/zoo
export HSA_ENABLE_IPC_MODE_LEGACY=0
S=8192x768x3072,8192x1024x4096,8192x1280x5120,8192x1792x6400,8192x3072x768,8192x4096x1024,8192x4096x14336,8192x5120x1280,8192x6400x1792,8192x8192x28672,8192x14336x4096,8192x28672x8192
for d in bf16 fp8; do
  timeout -k 10 400 python -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --rounds 5 --shapes $S > gpurun_out/zoo/$d.txt 2>&1 || exit $?
done
grep -h '^{' gpurun_out/zoo/*.txt
