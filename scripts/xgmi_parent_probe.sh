# Does a GPU-initialised parent process (pytest + torch) change how the
# xgmi kernels of 2 child ranks sharing the GPU behave? Control vs torch parent.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=10 DLNB_COMMTEST_VERBOSE=1 DLNB_XGMI_REGION_MB=1 DLNB_XGMI_P2P_MB=1
CMD="python -m dlnetbench_amd.utils.launch -n 2 --timeout 100 build/bin/dlnb commtest --backend xgmi -d 0,0 --sizes 1,7,100,4097,65536,300007,1048583"
timeout -k 10 110 $CMD > gpurun_out/probe_control.log 2>&1
echo "control rc=$?" >> gpurun_out/probe_steps.log
timeout -k 10 130 python -c "
import subprocess, sys, torch
assert torch.cuda.is_available()
sys.exit(subprocess.call('$CMD', shell=True))
" > gpurun_out/probe_torchparent.log 2>&1
echo "torchparent rc=$?" >> gpurun_out/probe_steps.log
