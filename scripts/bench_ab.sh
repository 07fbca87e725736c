# A/B of the compute-stream boundary costs at N=1 (llama3_8b FSDP bench).
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ab() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/ab_$name.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["exposed_comm_ms"])' 2>/dev/null)" >> gpurun_out/ab_steps.log
  [ $rc -eq 0 ] || exit $rc
}
ab default DLNB_X=0
ab nostall DLNB_STALL_TIMERS=0
ab slice2ms DLNB_GEMM_SLICE_US=2000

timeout -k 10 200 python bench.py --steps 3 --warmup 1 --compute sleep > gpurun_out/ab_sleep.log 2>&1
echo "sleep rc=$? $(grep '^{' gpurun_out/ab_sleep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["exposed_comm_ms"])' 2>/dev/null)" >> gpurun_out/ab_steps.log
