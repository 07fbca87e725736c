"""Round 5: pipeline stall timers from task stamps (TimerSet::stall_before_task) - per rank, the iteration over
its compute floor against the sum of its exposed-wait timers (hybrid_3d S=2, loopback ranks on one GPU)."""
import json
import sys

from dlnetbench_amd import engine

out = {}
for compute in ("sleep", "gemm"):
    for stamps in ("1", "0"):
        doc = engine.run_native("hybrid_3d", "tiny_dense_8_bfloat16", 2, 8, 1, base_path="tests/data", warmup=2, runs=5,
                         compute=compute, backend="loopback", ranks=2, quiet=True, env={"DLNB_TASK_STAMP_TIMERS": stamps})
        g = doc["global"]
        row = {"median_ms": g["dlnb"]["iteration"]["median_ms"], "floor_ms": g["dlnb"]["iteration"]["compute_floor_ms"],
               "ranks": []}
        for r in doc["ranks"]:
            keys = {k: v for k, v in r.items() if isinstance(v, list) and v and isinstance(v[0], (int, float))}
            row["ranks"].append({k: [round(sum(v) / 5 * 1e3, 4), len(v)] for k, v in keys.items()})
        out[f"{compute}_stamps{stamps}"] = row
        print(compute, stamps, json.dumps(row), flush=True)
json.dump(out, open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pp_timers.json", "w"), indent=1)
