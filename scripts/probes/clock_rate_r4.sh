#!/bin/bash
# Round 4: the deadline clock's rate against the host clock.
#   1. scripts/probes/src/clock_rate.hip (built to build/bin/probe_clock_rate): readings over 0.5..15.5 s windows
#   2. clock_check --long-ms 2000: host time of 2-s idle waits with the measured rate (default, 0.5-s window),
#      a 3-s window, and the nominal 100 MHz (DLNB_CLOCK_CAL_MS=0), interleaved
set -u
O=gpurun_out/clock
mkdir -p $O
C="python -m dlnetbench_amd.tools.clock_check --long-ms 2000 --reps 5"
timeout -k 10 60 build/bin/probe_clock_rate > $O/probe.txt 2>&1 &&
timeout -k 10 120 $C > $O/measured.json 2> $O/measured.err &&
DLNB_CLOCK_CAL_MS=0 timeout -k 10 120 $C > $O/nominal.json 2> $O/nominal.err &&
DLNB_CLOCK_CAL_MS=3000 timeout -k 10 120 $C > $O/measured3s.json 2> $O/measured3s.err &&
timeout -k 10 120 $C > $O/measured2.json 2> $O/measured2.err &&
echo done >> $O/steps.log
