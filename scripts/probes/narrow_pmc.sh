# PMC of the narrow-tile fp8 / bf16 GEMM next to hipBLASLt at the C5 stand-in shape 8192 x 1280 x 5120 (one pass of
# SQ / GRBM counters per dtype; each pass under its own time limit). Output: gpurun_out/npmc_{fp8,bf16}/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
for d in fp8 bf16; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/npmc_$d -o g -- python3 -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --shapes 8192x1280x5120 --rounds 2 --iters 5 > gpurun_out/npmc_$d.log 2>&1
  python -m dlnetbench_amd.tools.prof_summary --pmc gpurun_out/npmc_$d --title "PMC $d 8192x1280x5120" > gpurun_out/npmc_$d.md
done
cat gpurun_out/npmc_*.md
