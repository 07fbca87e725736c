#!/bin/bash
# dp vit_h_32_float8 (8 buckets, graph) at few vs many iterations, fp8 4-wave vs 8-phase deadline kernel.
set -u
mkdir -p gpurun_out
for k in 1 0; do
  for wr in "1 2" "5 20"; do
    set -- $wr
    DLNB_GEMM_FP8_DL_4WAVE=$k timeout -k 10 120 build/bin/dp vit_h_32_float8 8 . --no-topology --quiet -w $1 -r $2 --graph \
      --json gpurun_out/vw.json > gpurun_out/vw.log 2>&1 || exit $?
    python3 -c "import json; d=json.load(open('gpurun_out/vw.json'))['global']['dlnb']['iteration']; print('4wave=$k w=$1 r=$2', round(d['timed_ms_per_iter'],3), round(d['median_ms'],3), [round(x,3) for x in d.get('iteration_ms', [])][:20] if 'iteration_ms' in d else '')"
  done
done
