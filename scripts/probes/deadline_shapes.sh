#!/bin/bash
# The deadline GEMM at the FFN up-projection shape (K = hidden, the stand-in of
# rounds 1-2) and at the down-projection shape (K = ffn): PMC per clock, one-shot
# and deadline, via deadline_pmc.sh.
set -u
for s in "8192 14336 4096" "8192 4096 14336"; do
  tag=$(echo $s | tr ' ' x)
  SHAPE="$s" bash scripts/probes/deadline_pmc.sh || exit 1
  mv gpurun_out/deadline_pmc gpurun_out/deadline_pmc_$tag
done
