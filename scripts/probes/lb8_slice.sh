# Loopback 8-rank FSDP / hybrid_3d rehearsal with 500-us deadline slices (the round-2 default) vs one launch per
# task (round 3): does slicing explain the slower loopback medians? Output: gpurun_out/lb8s_*.json.
set -u
export HSA_ENABLE_IPC_MODE_LEGACY=0
for sl in 500 0; do
  DLNB_GEMM_SLICE_US=$sl timeout -k 10 240 build/bin/fsdp llama3_8b_16_bfloat16 32 8 . --backend loopback --ranks 8 -w 1 -r 2 --quiet --no-topology --time-scale 0.05 --json gpurun_out/lb8s_fsdp_$sl.json > /dev/null 2>&1 || exit $?
  DLNB_GEMM_SLICE_US=$sl timeout -k 10 300 build/bin/hybrid_3d llama3_70b_16_bfloat16 2 4 4 . --backend loopback --ranks 8 -w 1 -r 2 --quiet --no-topology --time-scale 0.02 --in-place --json gpurun_out/lb8s_h3d_$sl.json > /dev/null 2>&1 || exit $?
done
python3 - <<'PY'
import json
for n in ("fsdp", "h3d"):
    for sl in (500, 0):
        d = json.load(open(f"gpurun_out/lb8s_{n}_{sl}.json"))
        print(n, sl, round(d["global"]["dlnb"]["iteration"]["median_ms"], 1))
PY
