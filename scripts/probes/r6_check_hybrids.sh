# Round 6: the hybrids' TP / EP placement (inner lane under lane graphs, compute stream otherwise) on the GPU:
# the 2-rank lane tests, the timer value tests, the 4-rank bench rehearsal.
set -u
bash scripts/probes/gpu_steps.sh gpurun_out/r6i "500 strat.log tests/test_gpu_strategies.py --timeout 200 -k two_ranks+or+pipeline+or+hybrid+or+optimizer" \
  "500 timers.log tests/test_gpu_timers.py --timeout 300 -k tp_+or+ep_+or+pipeline" || exit $?
timeout -k 10 300 python -u scripts/probes/hyb_n4_ab_r6.py c3 > gpurun_out/r6i/hyb_c3.log 2>&1 &&
timeout -k 10 300 python -u scripts/probes/hyb_n4_ab_r6.py c4 > gpurun_out/r6i/hyb_c4.log 2>&1 &&
bash scripts/probes/bench_n4_one_gpu.sh
