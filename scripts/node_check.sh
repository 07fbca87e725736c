#!/bin/bash
# Multi-GPU node check (run on an 8 x MI355X node; not part of the 1-GPU CI):
# exact collectives over every backend across all visible GPUs, then the
# nccl-tests style bandwidth tables for RCCL and the xgmi kernels (staged and
# zero-copy registered), graph-replayed. Each step has its own time limit and
# the script stops at the first failure.
#   scripts/node_check.sh [N]        (default: all visible GPUs)
set -u
N=${1:-$(python3 -c "import ctypes,sys; sys.path.insert(0,'.'); from dlnetbench_amd import _native as n; print(n.lib().dlnb_gpu_count())")}
mkdir -p gpurun_out/node_check
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=${DLNB_XGMI_TIMEOUT_S:-30}
L="python -m dlnetbench_amd.utils.launch -n $N --timeout 280"
step() {  # name args...
  local name=$1; shift
  echo "=== $name: $*"
  timeout -k 10 300 $L build/bin/dlnb commtest "$@" > gpurun_out/node_check/$name.log 2> gpurun_out/node_check/$name.err
  local rc=$?
  grep '^{' gpurun_out/node_check/$name.log | head -3
  [ $rc -eq 0 ] || { echo "$name failed (rc=$rc), see gpurun_out/node_check/$name.err"; exit $rc; }
}
step rccl_check --backend rccl
step xgmi_check --backend xgmi
step xgmi_check_graph_registered --backend xgmi --graph --registered
step mixed_check --backend mixed
step rccl_bench --backend rccl --bench --graph
step xgmi_bench --backend xgmi --bench --graph
step xgmi_bench_registered --backend xgmi --bench --graph --registered
echo "all steps passed; tables: gpurun_out/node_check/*_bench*.log"
