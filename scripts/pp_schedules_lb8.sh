# Pipeline schedules side by side: hybrid_2d llama3_8b, S=8 stages x mb=16
# microbatches as 8 rank threads on ONE MI355X (--backend loopback), compute
# = the idle-wait kernel (--compute sleep) so the 8 ranks' compute overlaps as
# on 8 GPUs and the schedule's bubble is what the timings show.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" build/bin/hybrid_2d llama3_8b_16_bfloat16 8 16 . --backend loopback --ranks 8 -w 1 -r 3 \
    --quiet --no-topology --compute sleep --json gpurun_out/pp_${name}.json "$@" > gpurun_out/pp_${name}.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/pp_steps.log
  [ $rc -eq 0 ] || exit $rc
}
run gpipe 120 --pp-schedule gpipe
run 1f1b 120 --pp-schedule 1f1b
run interleaved2 120 --pp-schedule interleaved --pp-virtual 2
run dualpipe 120 --pp-schedule dualpipe
