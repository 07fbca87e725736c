# Every strategy at W=1 on the real model tables: eager enqueue vs HIP graph.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {  # name args...
  local name=$1; shift
  for g in "" "--graph"; do
    timeout -k 10 300 build/bin/"$@" . -w 1 -r 2 --quiet --no-topology $g --json gpurun_out/w1_${name}${g:+_graph}.json \
      > gpurun_out/w1_${name}${g:+_graph}.log 2>&1
    local rc=$?
    echo "$name $g rc=$rc" >> gpurun_out/w1_steps.log
    [ $rc -eq 0 ] || exit $rc
  done
}
run dp_vit_h_fp8 dp vit_h_32_float8 8
run dp_gpt2_l dp gpt2_l_16_bfloat16 4
run fsdp_llama3_8b fsdp llama3_8b_16_bfloat16 32 1
run h2d_llama3_8b hybrid_2d llama3_8b_16_bfloat16 1 4
run h3d_llama3_8b hybrid_3d llama3_8b_16_bfloat16 1 4 1
run h3d_1f1b_llama3_8b hybrid_3d llama3_8b_16_bfloat16 1 4 1 --pp-schedule 1f1b
run moe_mixtral_scaled hybrid_3d_moe mixtral_8x7b_16_bfloat16 1 4 1 --time-scale 0.1
# extensions
run dpz2_llama3_8b dp llama3_8b_16_bfloat16 10 --zero 2
run cp_llama3_8b hybrid_cp llama3_8b_16_bfloat16 1
run h3d_sp_llama3_8b hybrid_3d llama3_8b_16_bfloat16 1 4 1 --sequence-parallel
run h4d_mixtral_scaled hybrid_4d mixtral_8x7b_16_bfloat16 1 4 1 1 --time-scale 0.1
