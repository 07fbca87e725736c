# xgmi backend debugging on one GPU: N ranks on device 0, per-size timings,
# optional flag dumps after every kernel (arg 3 = 1), short device timeout.
set -u
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=${DLNB_XGMI_TIMEOUT_S:-8} DLNB_COMMTEST_VERBOSE=1
sizes=${1:-1,7,100,4097,65536,300007,1048583}
n=${2:-2}
debug=${3:-0}
devs=$(python3 -c "print(','.join(['0']*$n))")
DLNB_XGMI_DEBUG=$debug DLNB_XGMI_REGION_MB=1 DLNB_XGMI_P2P_MB=1 timeout -k 10 200 python -m dlnetbench_amd.utils.launch -n $n --timeout 190 build/bin/dlnb commtest --backend xgmi -d $devs --sizes $sizes > gpurun_out/dbg.log 2>&1
echo "rc=$?" >> gpurun_out/dbg_steps.log
