# Round-6 final check: the GPU suite, the timer value tests, smoke(), a driver-style 20-step bench line (each
# bounded; a failing test does not stop the later steps, a time limit or crash does).
set -u
mkdir -p gpurun_out/r6end
bash scripts/probes/gpu_steps.sh gpurun_out/r6end "900 suite.log tests -m gpu --timeout 300 --deselect tests/test_gpu_timers.py" \
  "600 timers.log tests/test_gpu_timers.py --timeout 300"
rc=$?
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r6end/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py --steps 20 --warmup 1 > gpurun_out/r6end/bench.log 2> gpurun_out/r6end/bench.err
