# The BASELINE.json 8-GPU configs as 8 rank threads on ONE MI355X (--backend
# loopback): full-size messages and per-rank memory, compute scaled down.
# Functional rehearsal of the W=8 paths; timings are not xGMI timings.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name timeout args...
  local name=$1 to=$2; shift 2
  timeout -k 10 "$to" build/bin/"$@" . --backend loopback --ranks 8 -w 1 -r 2 --quiet --no-topology \
    --json gpurun_out/lb8_${name}.json > gpurun_out/lb8_${name}.log 2>&1
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/lb8_steps.log
  [ $rc -eq 0 ] || exit $rc
}
run fsdp_llama3_8b 240 fsdp llama3_8b_16_bfloat16 32 8 --time-scale 0.05
run dp_vit_h_fp8 240 dp vit_h_32_float8 8
run h3d_llama3_70b 300 hybrid_3d llama3_70b_16_bfloat16 2 4 4 --time-scale 0.02 --in-place
run moe_mixtral 300 hybrid_3d_moe mixtral_8x7b_16_bfloat16 2 16 4 --time-scale 0.02 --in-place
