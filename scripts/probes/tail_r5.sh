#!/bin/bash
# Round 5: the headline's occasional slow tail (barrier 0.36 instead of 0.19 ms in ~3 of 20 runs): a kernel trace
# of 12 full-scale FSDP iterations (lane graphs), plus the same run untraced with per-run timers.
set -u
O=${O:-gpurun_out/tail}
mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_NO_TORCH=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
H="build/bin/fsdp llama3_8b_16_bfloat16 32 1 . --backend rccl --compute gemm --graph --quiet --silent -w 2 -r 12"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o h -- $H --json $O/traced.json > $O/trace.log 2>&1 \
  && timeout -k 10 200 $H --json $O/plain.json > $O/plain.log 2>&1
echo "rc=$?" > $O/done.txt
