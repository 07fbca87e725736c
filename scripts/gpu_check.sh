#!/bin/bash
# GPU session driver: each step under its own timeout; stop at the first
# timeout / abort / segfault (never retry a failing GPU step).
# usage: scripts/gpu_check.sh <step>...   steps: pytest bench benchvariants prof
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name: $*" >> gpurun_out/steps.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" >> gpurun_out/steps.log
  case $rc in
    0|1) return 0 ;;        # pass / test failures: keep going
    *) echo "fatal rc=$rc in $name, stopping" >> gpurun_out/steps.log; exit $rc ;;
  esac
}
for step in "$@"; do
  case $step in
    pytest) run pytest_gpu 900 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 170 --timeout-method thread ;;
    loopback) run loopback_gpu 600 python -u -m pytest tests/test_gpu_strategies.py -m gpu -v -k loopback -p no:cacheprovider --timeout 170 --timeout-method thread ;;
    bench) run bench 300 python bench.py --steps 3 --warmup 1 --json gpurun_out/bench_report.json ;;
    benchdriver) run bench_driver 400 python bench.py --steps 20 --warmup 5 --json gpurun_out/bench_driver_report.json ;;
    clock) run clock 120 python -m dlnetbench_amd.tools.clock_check ;;
    hwmon) run hwmon 30 bash -c "ls -la /sys/class/drm/card*/device/hwmon/hwmon*/ | head -80" ;;
    benchvariants)
      run bench_gemmwork 300 python bench.py --steps 2 --warmup 1 --compute gemm-work
      run bench_sleep 300 python bench.py --steps 2 --warmup 1 --compute sleep
      run bench_reference 300 python bench.py --steps 2 --warmup 1 --schedule reference ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      run prof_fsdp 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fsdp -o fsdp -- python3 bench.py --steps 1 --warmup 1 ;;
    gemmbench)
      run gemmbench_bf16 300 python -m dlnetbench_amd.tools.gemm_bench --dtype bf16
      run gemmbench_fp8 300 python -m dlnetbench_amd.tools.gemm_bench --dtype fp8 --shapes 4096x4096x4096,8192x8192x8192,8192x14336x4096 ;;
    pmcfsdp)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      # counter collection serialises dispatches: eager enqueue, 20 ms slices
      run pmc_fsdp 400 env DLNB_GEMM_SLICE_US=20000 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmc_fsdp -o fsdp -- python3 bench.py --steps 1 --warmup 0 --no-graph ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      run pmc_gemm 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_gemm -o gemm -- python3 -m dlnetbench_amd.tools.gemm_bench --shapes 8192x14336x4096 --rounds 2 --iters 5 ;;
    xgmi)
      run xgmi_w2 150 env DLNB_COMMTEST_VERBOSE=1 DLNB_XGMI_TIMEOUT_S=10 DLNB_XGMI_REGION_MB=1 DLNB_XGMI_P2P_MB=1 python -m dlnetbench_amd.utils.launch -n 2 --timeout 120 build/bin/dlnb commtest --backend xgmi -d 0,0
      run xgmi_w4 150 env DLNB_COMMTEST_VERBOSE=1 DLNB_XGMI_TIMEOUT_S=10 python -m dlnetbench_amd.utils.launch -n 4 --timeout 120 build/bin/dlnb commtest --backend xgmi -d 0,0,0,0
      run xgmi_bench 200 env DLNB_XGMI_TIMEOUT_S=30 python -m dlnetbench_amd.utils.launch -n 2 --timeout 180 build/bin/dlnb commtest --backend xgmi -d 0,0 --bench --sizes 1024,65536,1048576,16777216,67108864
      run rccl_bench 200 build/bin/dlnb commtest --backend rccl --bench --sizes 1024,65536,1048576,16777216,67108864 ;;
    dp8) run bench_dp 300 python -m dlnetbench_amd.tools.sweep --quick ;;
    counters)
      # bench headline (FSDP, N = 1) with rocprof counters folded into its report (global.dlnb.counters):
      # a kernel trace of the graph-replayed run + two PMC passes (TCC holds FETCH_SIZE or WRITE_SIZE, not
      # both) of one eagerly enqueued iteration (one deadline launch per task, the default).
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      B="bench.py --c5-model none --stretch-steps 0"
      run cnt_trace 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/cnt_trace -o bench -- python3 $B --steps 2 --warmup 1 --json gpurun_out/bench_cnt_report.json
      run cnt_pmc_a 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 FETCH_SIZE --output-format csv -d gpurun_out/cnt_pmc_a -o a -- python3 $B --steps 1 --warmup 0 --no-graph
      run cnt_pmc_b 400 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/cnt_pmc_b -o b -- python3 $B --steps 1 --warmup 0 --no-graph
      run cnt_merge 60 python -m dlnetbench_amd.tools.prof_merge gpurun_out/bench_cnt_report.json gpurun_out/cnt_trace gpurun_out/cnt_pmc_a gpurun_out/cnt_pmc_b -o gpurun_out/bench_counters.json ;;
    *) echo "unknown step $step" >> gpurun_out/steps.log ;;
  esac
done
