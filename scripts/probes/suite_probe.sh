set -u
mkdir -p gpurun_out/suite_probe
export HSA_ENABLE_IPC_MODE_LEGACY=0 DLNB_XGMI_TIMEOUT_S=30
timeout -k 10 150 python -m dlnetbench_amd.utils.launch -n 2 --timeout 130 build/bin/dlnb commtest --suite --backends xgmi -d 0,0 --dtypes bf16,fp8_e4m3 --json gpurun_out/suite_probe/xgmi2.json > gpurun_out/suite_probe/xgmi2.log 2>&1 &&
timeout -k 10 150 python -m dlnetbench_amd.utils.launch -n 1 --timeout 130 build/bin/dlnb commtest --suite --backends rccl --dtypes bf16,fp8_e4m3 --json gpurun_out/suite_probe/rccl1.json > gpurun_out/suite_probe/rccl1.log 2>&1 &&
rm -f gpurun_out/xgmi_sweep.jsonl && timeout -k 10 500 bash scripts/xgmi_sweep.sh 2 uncached "256" && cp gpurun_out/xgmi_sweep.jsonl gpurun_out/suite_probe/sweep_staged.jsonl &&
rm -f gpurun_out/xgmi_sweep.jsonl && EXTRA=--registered timeout -k 10 500 bash scripts/xgmi_sweep.sh 2 uncached "256" && cp gpurun_out/xgmi_sweep.jsonl gpurun_out/suite_probe/sweep_reg.jsonl
