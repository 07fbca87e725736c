#!/bin/bash
# Tile-order group size (DLNB_GEMM_GROUP M-tiles per L2 group) for the fp8 4-wave GEMM.
for g in ${GROUPS_:-4 8 16 32}; do
  echo "GROUP=$g"
  DLNB_GEMM_GROUP=$g timeout -k 10 100 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --variants 5 \
    --shapes 8192x14336x4096,8192x8192x8192 || exit 1
done
