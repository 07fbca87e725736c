#!/bin/bash
# Deadline GEMM: per-tile persistent loop (DLNB_GEMM_STREAM=0) vs the streaming
# kernel (1), bf16 / fp8, llama3-8B FFN shape and ViT-H FFN shape (K = 1280).
# Summary: python scripts/probes/deadline_stream_table.py gpurun_out/dstream
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/dstream
SHAPES=${SHAPES:-"8192 14336 4096|8192 5120 1280"}
DTS=${DTS:-"bf16 fp8"}
VARIANTS=${VARIANTS:-"0 1"}
IFS="|" read -ra SH <<< "$SHAPES"
for shape in "${SH[@]}"; do
  for dt in $DTS; do
    for s in $VARIANTS; do
      tag="${dt}_$(echo $shape | tr ' ' x)_s$s"
      # s: 0 per-tile loop (tail instantiations), 1 streaming kernel, 2 per-tile with one uniform K-tile body (fp8)
      case $s in 0) ev="DLNB_GEMM_STREAM=0 DLNB_GEMM_FP8_DL_UNIFORM=0" ;; 1) ev="DLNB_GEMM_STREAM=1" ;;
                 2) ev="DLNB_GEMM_STREAM=0 DLNB_GEMM_FP8_DL_UNIFORM=1" ;; esac
      env $ev timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_VALU_MFMA_MOPS_F8 \
        SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/dstream/$tag -o r \
        -- python3 scripts/probes/deadline_stream.py $dt $shape > gpurun_out/dstream/$tag.log 2>&1 || exit $?
    done
  done
done
