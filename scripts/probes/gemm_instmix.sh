#!/bin/bash
# Instruction mix of our square GEMMs vs the vendor's at the headline stand-in shape (same MFMA
# cycles, lower clock under the power cap for bf16 -> what else do our waves execute per MFMA?). One 8-counter
# pass per dtype (7 SQ + GRBM), over gemm_bench's interleaved rounds. Output: gpurun_out/instmix_<dtype>/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export HSA_ENABLE_IPC_MODE_LEGACY=0
SHAPES=${SHAPES:-8192x4096x14336}
for d in ${DTYPES:-bf16 fp8}; do
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM SQ_INSTS_MFMA SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/instmix_$d -o g -- python3 -m dlnetbench_amd.tools.gemm_bench --dtype $d --variants 0 --shapes $SHAPES --rounds 2 --iters 5 > gpurun_out/instmix_$d.log 2>&1 || exit $?
done
echo done > gpurun_out/instmix_done.txt
# the headline's iteration boundary on the device clock (host spans in the timeline)
mkdir -p gpurun_out/tlhost
DLNB_NO_TORCH=1 timeout -k 10 150 build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph -w 1 -r 3 \
  --quiet --silent --timeline gpurun_out/tlhost/tl.json > gpurun_out/tlhost/run.log 2>&1 &&
python -m dlnetbench_amd timeline gpurun_out/tlhost/tl.json --check > gpurun_out/tlhost/summary.txt 2>&1
