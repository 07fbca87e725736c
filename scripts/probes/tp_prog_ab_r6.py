"""hybrid_3d 1 4 2 (T = 2) on two ranks sharing GPU 0: lane graphs with the compute program (default), lane
graphs with one launch per task (DLNB_COMPUTE_PROGRAMS=0), the single graph (DLNB_LANE_GRAPHS=0); medians
and the TP timers, 2 interleaved rounds."""
import json
import os
import pathlib
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_strategies import _two_ranks_one_gpu  # noqa: E402

params = sys.argv[1].split(",") if len(sys.argv) > 1 else ["1", "4", "2"]
ctas = int(sys.argv[2]) if len(sys.argv) > 2 else 8
variants = {"prog": {}, "noprog": {"DLNB_COMPUTE_PROGRAMS": "0"}, "single": {"DLNB_LANE_GRAPHS": "0"}}
out = {}
for rnd in range(2):
    for name, env in variants.items():
        tmp = pathlib.Path(tempfile.mkdtemp())
        d = _two_ranks_one_gpu(ROOT, tmp, "hybrid_3d", params, env, iters=8, ctas=ctas)
        g = d["global"]["dlnb"]
        r0 = [r for r in d["ranks"] if r.get("rank", 0) == 0][0]
        per = len(r0["runtimes"])
        res = {"median_ms": round(g["iteration"]["median_ms"], 3), "floor_ms": round(g["iteration"]["compute_floor_ms"], 3),
               "lanes": g["lane_graphs"].get("enabled"), "join": g["lane_graphs"].get("program_join"),
               "tp_comm_ms_per_iter": round(sum(r0.get("tp_comm_time", [])) / per * 1e3, 3),
               "tp_ar_ms_per_iter": round(sum(r0.get("tp_ar_time", [])) / per * 1e3, 3)}
        out.setdefault(name, []).append(res)
        print(rnd, name, json.dumps(res), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out", "r6g"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "r6g", "tp_prog_ab_" + "_".join(params) + f"_c{ctas}.json"), "w"), indent=1)
