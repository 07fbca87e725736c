# Program-mode 8-phase kernel throughput (the fixed-work calibration's round: compute.fixed_work.tflops) per
# tile-order group (DLNB_DEADLINE_GROUP), two interleaved rounds.
set -u
mkdir -p gpurun_out/r6z
for rnd in ${RNDS:-1 2}; do for g in ${GROUPS_AB:-4 8 16 32}; do
  DLNB_DEADLINE_GROUP=$g timeout -k 10 120 ./build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --no-topology --compute gemm-work \
    --backend rccl --graph -w 1 -r 2 --time-scale 0.05 --quiet --json gpurun_out/r6z/g$g.$rnd.json > gpurun_out/r6z/g$g.$rnd.log 2>&1 || exit 1
done; done
