"""Robustness sweep: every strategy family on two ranks sharing GPU 0 over xgmi with lane graphs allowed
(DLNB_LANE_SHARED=1), eager / --graph, gemm and gemm-work compute, with and without --optimizer; each job
bounded (40 s). Prints one line per configuration: ok / failure, lanes, join, timeouts, median vs floor."""
import json
import os
import pathlib
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_strategies as t  # noqa: E402

DATA = os.path.join(ROOT, "tests", "data")
L = "llama3_8b_16_bfloat16"
configs = [
    ("dp", "vit_h_32_float8", ["8"], ROOT, ()),
    ("dp", "vit_h_32_float8", ["8"], ROOT, ("--zero", "1", "--wire-dtype", "bf16")),
    ("dp", "vit_h_32_float8", ["8"], ROOT, ("--zero", "2", "--wire-dtype", "bf16")),
    ("dp", "vit_h_32_float8", ["8"], ROOT, ("--optimizer", "--wire-dtype", "bf16")),
    ("fsdp", L, ["32", "2"], ROOT, ()),
    ("fsdp", L, ["32", "2"], ROOT, ("--optimizer",)),
    ("fsdp", L, ["32", "1"], ROOT, ()),
    ("hybrid_2d", L, ["2", "4"], ROOT, ("--pp-schedule", "1f1b", "--optimizer")),
    ("hybrid_2d", L, ["2", "8"], ROOT, ("--pp-schedule", "interleaved", "--pp-virtual", "4")),
    ("hybrid_3d", L, ["2", "4", "1"], ROOT, ("--dp-buckets", "4")),
    ("hybrid_3d", L, ["1", "4", "2"], ROOT, ("--sequence-parallel",)),
    ("hybrid_3d_moe", "slow_moe_8_bfloat16", ["1", "8", "2"], DATA, ("--ep-overlap",)),
    ("hybrid_3d_moe", "slow_moe_8_bfloat16", ["2", "8", "1"], DATA, ()),
    ("hybrid_cp", L, ["2"], ROOT, ("--cp-algo", "ring")),
    ("hybrid_cp", L, ["2"], ROOT, ("--cp-algo", "ulysses")),
    ("hybrid_4d", "tiny_moe_8_bfloat16", ["1", "2", "1", "2"], DATA, ()),
]
computes = sys.argv[1].split(",") if len(sys.argv) > 1 else ["gemm"]
for binary, model, params, base, extra in configs:
    for compute in computes:
        tmp = pathlib.Path(tempfile.mkdtemp())
        tag = f"{binary} {' '.join(params)} {' '.join(extra)} [{compute}]"
        ts = "1" if base == DATA and model.startswith("slow") else "0.05"
        try:
            d = t._two_ranks_one_gpu(ROOT, tmp, binary, params, {"DLNB_GATE_TIMEOUT_S": "10"}, iters=3, model=model,
                                     time_scale=ts, base=base, extra_args=extra + (("--compute", compute) if compute != "gemm" else ()))
            g = d["global"]["dlnb"]
            lg = g.get("lane_graphs") or {}
            cc = g.get("chain_capped") or {}
            neg = [r.get("timer_negative_intervals") for r in d["ranks"] if r.get("timer_negative_intervals")]
            print("OK  ", tag, json.dumps({"median": round(g["iteration"]["median_ms"], 2),
                                           "floor": round(g["iteration"]["compute_floor_ms"], 2),
                                           "lanes": lg.get("enabled"), "join": lg.get("program_join"),
                                           "reason": (lg.get("reason") or "")[:60],
                                           "gto": cc.get("gate_wait_timeouts_max"), "cgto": cc.get("compute_gate_timeouts_max"),
                                           "neg": neg}), flush=True)
        except Exception as e:  # noqa: BLE001
            print("FAIL", tag, str(e)[:500].replace("\n", " | "), flush=True)
