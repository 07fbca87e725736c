# A/B of bench.py variants at N=1 (llama3_8b FSDP): one bench per variant,
# each under its own limit; results appended to gpurun_out/ab_steps.log.
#   scripts/bench_ab.sh default nostall graph sleep slice2ms
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for v in "$@"; do
  case $v in
    default) args=(); envs=(DLNB_X=0) ;;
    nostall) args=(); envs=(DLNB_STALL_TIMERS=0) ;;
    slice2ms) args=(); envs=(DLNB_GEMM_SLICE_US=2000) ;;
    graph) args=(--graph); envs=(DLNB_X=0) ;;
    graph_nostall) args=(--graph); envs=(DLNB_STALL_TIMERS=0) ;;
    sleep) args=(--compute sleep); envs=(DLNB_X=0) ;;
    *) echo "unknown variant $v" >> gpurun_out/ab_steps.log; continue ;;
  esac
  env "${envs[@]}" timeout -k 10 240 python bench.py --steps 3 --warmup 1 "${args[@]}" > gpurun_out/ab_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(grep '^{' gpurun_out/ab_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["exposed_comm_ms"])' 2>/dev/null)" >> gpurun_out/ab_steps.log
  [ $rc -eq 0 ] || exit $rc
done
