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
    pytest) run pytest_gpu 600 python -m pytest tests -m gpu -q -p no:cacheprovider ;;
    bench) run bench 300 python bench.py --steps 3 --warmup 1 ;;
    benchvariants)
      run bench_gemmwork 300 python bench.py --steps 2 --warmup 1 --compute gemm-work
      run bench_sleep 300 python bench.py --steps 2 --warmup 1 --compute sleep
      run bench_reference 300 python bench.py --steps 2 --warmup 1 --schedule reference ;;
    prof)
      cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
      run prof_fsdp 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fsdp -o fsdp -- python3 bench.py --steps 1 --warmup 1 ;;
    *) echo "unknown step $step" >> gpurun_out/steps.log ;;
  esac
done
