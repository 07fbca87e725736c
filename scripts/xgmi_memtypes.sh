# xgmi window memory type A/B (2 ranks on GPU 0): exact check + bandwidth.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=20
for mem in uncached fine coarse; do
  DLNB_XGMI_MEM=$mem timeout -k 10 150 python -m dlnetbench_amd.utils.launch -n 2 --timeout 140 build/bin/dlnb commtest \
    --backend xgmi -d 0,0 > gpurun_out/mem_$mem.check 2>&1
  echo "$mem check rc=$? $(grep '^{' gpurun_out/mem_$mem.check)" >> gpurun_out/mem_steps.log
  DLNB_XGMI_MEM=$mem timeout -k 10 150 python -m dlnetbench_amd.utils.launch -n 2 --timeout 140 build/bin/dlnb commtest \
    --backend xgmi -d 0,0 --bench --sizes 1048576,16777216,67108864 > gpurun_out/mem_$mem.bench 2>&1
  echo "$mem bench rc=$?" >> gpurun_out/mem_steps.log
done
