# Loopback 8-rank rehearsal of the BASELINE configs (scripts/loopback_w8.sh) + the loopback / xgmi GPU strategy
# tests, after ranks sharing a device default to 500-us deadline slices.
set -o pipefail
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest tests/test_gpu_strategies.py -m gpu -v -k "loopback or xgmi" -p no:cacheprovider --timeout 170 --timeout-method thread > gpurun_out/lb8_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/lb8_pytest.log; exit 1; }
tail -2 gpurun_out/lb8_pytest.log
bash scripts/loopback_w8.sh && python scripts/lb8_table.py > gpurun_out/lb8_table.md && cat gpurun_out/lb8_table.md
