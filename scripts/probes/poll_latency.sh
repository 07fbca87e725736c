#!/bin/bash
# Host wait latency per iteration: dp vit_h_32_float8 (8 buckets, graph), 5 warm-up + 50 timed iterations.
set -u
mkdir -p gpurun_out
timeout -k 10 120 build/bin/dp vit_h_32_float8 8 . --no-topology --quiet -w 5 -r 50 --graph --json gpurun_out/pl.json \
  > gpurun_out/pl.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/pl.json'))['global']['dlnb']['iteration']; print('vit graph', round(d['timed_ms_per_iter'],4), round(d['median_ms'],4))"
timeout -k 10 120 build/bin/dp gpt2_l_16_bfloat16 4 . --no-topology --quiet -w 5 -r 30 --graph --json gpurun_out/pl2.json \
  > gpurun_out/pl2.log 2>&1 || exit $?
python3 -c "import json; d=json.load(open('gpurun_out/pl2.json'))['global']['dlnb']['iteration']; print('gpt2 graph', round(d['timed_ms_per_iter'],4), round(d['median_ms'],4))"
