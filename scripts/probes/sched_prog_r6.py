"""hybrid_2d S=2 mb=4 on two ranks sharing GPU 0 (xgmi, lanes forced): each pipeline schedule with and
without the compute program; 60-s bound per job; prints the outcome and the lane info."""
import json
import os
import pathlib
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import test_gpu_strategies as t  # noqa: E402

scheds = sys.argv[1].split(",")
more = tuple(sys.argv[2].split()) if len(sys.argv) > 2 else ()
for sched in scheds:
    extra = json.loads(os.environ.get("XENV", "{}"))
    for name, env in (("prog", dict(extra)), ("noprog", {"DLNB_COMPUTE_PROGRAMS": "0"}))[:int(os.environ.get("NV", "3"))]:
        tmp = pathlib.Path(tempfile.mkdtemp())
        try:
            d = t._two_ranks_one_gpu(ROOT, tmp, "hybrid_2d", ["2", "4"], env, iters=4,
                                     extra_args=("--pp-schedule", sched) + more)
            g = d["global"]["dlnb"]
            print(sched, name, json.dumps({"median": round(g["iteration"]["median_ms"], 3),
                                           "floor": round(g["iteration"]["compute_floor_ms"], 3),
                                           "lanes": g["lane_graphs"].get("enabled"),
                                           "join": g["lane_graphs"].get("program_join"),
                                           "reason": g["lane_graphs"].get("reason"),
                                           "gto": g["chain_capped"]["gate_wait_timeouts_max"],
                                           "cgto": g["chain_capped"]["compute_gate_timeouts_max"],
                                           "program_tasks": g["compute"].get("program_tasks"),
                                           "programs": g["compute"].get("programs")}), flush=True)
        except AssertionError as e:
            print(sched, name, "FAILED", str(e)[:600], flush=True)
