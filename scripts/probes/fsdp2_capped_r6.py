"""FSDP U=32 F=2 on two ranks sharing GPU 0 (test_fsdp_lanes_two_ranks_one_gpu): chain_capped per variant."""
import json
import os
import pathlib
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_strategies import _two_ranks_one_gpu  # noqa: E402

variants = {"default": {}, "no_energy": {"DLNB_NO_ENERGY": "1"}, "no_task_stamps": {"DLNB_TASK_STAMP_TIMERS": "0"}}
for rnd in range(2):
    for name, env in variants.items():
        tmp = pathlib.Path(tempfile.mkdtemp())
        d = _two_ranks_one_gpu(ROOT, tmp, "fsdp", ["32", "2"], env)
        g = d["global"]["dlnb"]
        cc = g["chain_capped"]
        print(rnd, name, json.dumps({"median": round(g["iteration"]["median_ms"], 3),
                                     "floor": round(g["iteration"]["compute_floor_ms"], 3),
                                     "capped_tasks": cc["tasks_per_iter_max"], "capped_ms": cc["ms_per_iter_max"],
                                     "absorbed_ms": round(cc["absorbed_ms_per_iter_max"], 3),
                                     "gate_to": cc["gate_wait_timeouts_max"]}), flush=True)
