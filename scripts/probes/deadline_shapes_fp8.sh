#!/bin/bash
# fp8 (ViT-H/32: hidden 1280, FFN 5120): the deadline GEMM at the up- and the
# down-projection shape, PMC via deadline_pmc.sh.
set -u
for s in "8192 5120 1280 fp8" "8192 1280 5120 fp8"; do
  tag=$(echo $s | tr ' ' x)
  MOPS=F8 SHAPE="$s" bash scripts/probes/deadline_pmc.sh || exit 1
  mv gpurun_out/deadline_pmc gpurun_out/deadline_pmc_$tag
done
