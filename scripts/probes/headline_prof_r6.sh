# The headline step (FSDP llama3_8b U=32, lane graphs + compute program) under rocprofv3: a kernel-trace /
# stats pass and a separate PMC pass (MFMA work and busy cycles, GPU clock cycles).
set -u
out=gpurun_out/r6y
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
B="./build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --no-topology --compute gemm --backend rccl --graph -w 1 -r 3 --quiet"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o k -- $B --json $out/trace.json > $out/trace.log 2>&1 &&
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d $out/pmc -o p -- $B --json $out/pmc.json > $out/pmc.log 2>&1
