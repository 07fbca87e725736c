"""Per-entry exposed-communication timers of a base and a delayed run (DLNB_COMM_FAULT mode=delay), for
debugging tests/test_gpu_timers.py: prints every timer entry of the first timed iterations."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from dlnetbench_amd import engine  # noqa: E402


def show(tag, doc, keys, rank=0, n=40):
    r = doc["ranks"][rank]
    runs = len(r.get("runtimes") or r.get("runtime"))
    print(f"== {tag} rank {rank} runs {runs} median {doc['global']['dlnb']['iteration']['median_ms']:.3f} "
          f"lanes {doc['global']['dlnb'].get('lane_graphs', {}).get('enabled')}")
    for k in keys:
        v = [round(x * 1e3, 4) for x in r.get(k, [])]
        per = len(v) // max(1, runs)
        print(f"  {k}: {len(v)} entries ({per}/iter), sum/iter {sum(v) / max(1, runs):.4f} ms; first iter: {v[:per][:n]}")
    if "timer_negative_intervals" in r:
        print("  NEGATIVE", r["timer_negative_intervals"])


def one(strategy, model, params, mode, compute, fault, keys, time_scale=None, **kw):
    env = {"DLNB_COMM_FAULT": fault} if fault else {}
    if mode == "single":
        env["DLNB_LANE_GRAPHS"] = "0"
    d = engine.run_native(strategy, model, *params, base_path=ROOT, warmup=2, runs=4, compute=compute,
                          backend="rccl", graph=mode != "eager", time_scale=time_scale, quiet=True, env=env, **kw)
    show(f"{strategy} {mode} {compute} fault={bool(fault)}", d, keys)


if __name__ == "__main__":
    what = sys.argv[1]
    if what == "fsdp":
        U = 32
        fault = (f"mode=delay,us=500,op=all_gather,call=1,every={2 * U - 1};"
                 f"mode=delay,us=500,op=all_gather,call={U},every={2 * U - 1};"
                 f"mode=delay,us=500,op=reduce_scatter,call={U - 1},every={U}")
        for mode in sys.argv[2].split(","):
            for compute in sys.argv[3].split(","):
                for f in (None, fault):
                    one("fsdp", "llama3_8b_16_bfloat16", (U, 1), mode, compute, f,
                        ["allgather_wait_fwd", "allgather_wait_bwd", "barrier", "allgather_time"], time_scale=0.001)
    elif what in ("tp", "ep", "pp"):
        from test_gpu_timers import _two_ranks  # noqa: E402
        import pathlib
        import tempfile
        tmp = pathlib.Path(tempfile.mkdtemp())
        data = os.path.join(ROOT, "tests", "data")
        if what == "tp":
            fault = "mode=delay,us=500,op=all_reduce,comm=tp,call=0,every=16"
            args = ("hybrid_3d", "llama3_8b_16_bfloat16", (1, 4, 2))
            keys = ["tp_comm_time", "tp_ar_time"]
            ts, base = 0.05, ROOT
        elif what == "ep":
            fault = "mode=delay,us=500,op=all_to_all,comm=ep,call=0,every=128"
            args = ("hybrid_3d_moe", "slow_moe_8_bfloat16", (1, 8, 2))
            keys = ["ep_comm_time", "ep_a2a_time", "dp_ep_comm_time", "dp_exposed_time"]
            ts, base = 1.0, data
        else:
            fault = "mode=delay,us=500,op=send,rank=0,call=0,every=4"
            args = ("hybrid_2d", "llama3_8b_16_bfloat16", (2, 4))
            keys = ["pp_comm_time", "pp_send_time", "pp_recv_time"]
            ts, base = 0.02, ROOT
        for mode in sys.argv[2].split(","):
            for compute in sys.argv[3].split(","):
                for f in (None, fault):
                    d = _two_ranks(tmp, *args, mode, compute, f, ts, base=base)
                    for rank in (0, 1):
                        show(f"{args[0]} {mode} {compute} fault={bool(f)}", d, keys, rank=rank)
