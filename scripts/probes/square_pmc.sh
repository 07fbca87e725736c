# PMC of the square one-shot GEMMs next to hipBLASLt / _scaled_mm at the headline stand-in shape 8192 x 4096 x 14336
# (after the paired epilogue stores): one SQ / GRBM counter pass per dtype. Output: gpurun_out/spmc_{bf16,fp8}/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
for d in bf16 fp8; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/spmc_$d -o g -- python3 -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --shapes 8192x4096x14336 --rounds 2 --iters 5 > gpurun_out/spmc_$d.log 2>&1
  python -m dlnetbench_amd.tools.prof_summary --pmc gpurun_out/spmc_$d --title "PMC $d 8192x4096x14336" > gpurun_out/spmc_$d.md
done
cat gpurun_out/spmc_*.md
