# Every strategy at W = 1 on the real tables (time-scaled where long), --graph: lane graphs (default rule)
# against the single graph (DLNB_LANE_GRAPHS=0); one JSON per run under gpurun_out/r6u.
set -u
mkdir -p gpurun_out/r6u
run() {  # name binary args...
  local name=$1; shift
  for v in 1 0; do
    DLNB_LANE_GRAPHS=$v timeout -k 10 120 "$@" --no-topology --compute gemm --backend rccl --graph -w 2 -r 6 --quiet \
      --json gpurun_out/r6u/$name.$v.json > gpurun_out/r6u/$name.$v.log 2>&1 || return 1
  done
}
B=./build/bin
run dp $B/dp vit_h_32_float8 8 . &&
run zero1 $B/dp vit_h_32_float8 8 . --zero 1 --wire-dtype bf16 &&
run zero2 $B/dp vit_h_32_float8 8 . --zero 2 --wire-dtype bf16 &&
run fsdp $B/fsdp llama3_8b_16_bfloat16 32 1 . --time-scale 0.05 &&
run h2d $B/hybrid_2d llama3_8b_16_bfloat16 1 4 . --time-scale 0.05 &&
run h3d $B/hybrid_3d llama3_8b_16_bfloat16 1 4 1 . --time-scale 0.05 &&
run moe $B/hybrid_3d_moe slow_moe_8_bfloat16 1 8 1 tests/data --time-scale 0.2 &&
run cp $B/hybrid_cp llama3_8b_16_bfloat16 1 . --time-scale 0.05 &&
run h4d $B/hybrid_4d tiny_moe_8_bfloat16 1 2 1 1 tests/data
