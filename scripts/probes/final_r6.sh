# Round-6 final check: the GPU suite, the timer value tests, smoke(), a default bench line.
set -u
bash scripts/probes/gpu_steps.sh gpurun_out/r6k "900 suite.log tests -m gpu --timeout 300 --deselect tests/test_gpu_timers.py" \
  "600 timers.log tests/test_gpu_timers.py --timeout 300" || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6k/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/r6k/bench.log 2> gpurun_out/r6k/bench.err
