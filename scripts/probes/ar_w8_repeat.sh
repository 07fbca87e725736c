# 8 ranks sharing GPU 0, staged xgmi all-reduce at 16 Mi elements (graph-replayed), three separate jobs:
# is the 0.53 s outlier of release_ab (vmcnt) repeatable or a time-slicing artifact? Output: gpurun_out/ar8/.
set -u
mkdir -p gpurun_out/ar8
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=20 DLNB_XGMI_MEM=uncached DLNB_XGMI_BLOCKS=256
for i in 1 2 3; do
  timeout -k 10 120 python -m dlnetbench_amd.utils.launch -n 8 --timeout 100 build/bin/dlnb commtest --backend xgmi \
    -d 0,0,0,0,0,0,0,0 --bench --graph --iters 10 --warmup 3 --sizes 16777216 > gpurun_out/ar8/run$i.log 2> gpurun_out/ar8/run$i.err || exit $?
  grep '"all_reduce"' gpurun_out/ar8/run$i.log
done
