"""Python front-end for the native benchmark runtime.

``run("fsdp", "llama3_8b_16_bfloat16", 32, 8, base_path=".", warmup=1, runs=3)``
runs one rank of a benchmark in this process (rank identity comes from the
environment exactly like the CLI binaries) and returns the report document:
``{"section", "title", "global": {...}, "ranks": [{...}, ...]}`` with the
reference's key names plus ``global["dlnb"]`` extras.
"""
from __future__ import annotations

from typing import Any, Dict, List

from . import _native

POSITIONAL = {
    "dp": ["num_buckets"],
    "fsdp": ["num_units", "sharding_factor"],
    "hybrid_2d": ["num_stages", "num_microbatches"],
    "hybrid_3d": ["num_stages", "num_microbatches", "num_tensor_shards"],
    "hybrid_3d_moe": ["num_stages", "num_microbatches", "num_expert_shards"],
    "hybrid_cp": ["num_cp_shards"],
    "hybrid_4d": ["num_stages", "num_microbatches", "num_tensor_shards", "num_expert_shards"],
}

_FLAG = {
    "warmup": "-w", "runs": "-r", "devices": "-d", "min_exectime": "-m",
    "backend": "--backend", "compute": "--compute", "wire_dtype": "--wire-dtype",
    "compute_dtype": "--compute-dtype", "schedule": "--schedule", "tp_granularity": "--tp-granularity",
    "dp_buckets": "--dp-buckets", "max_loop_iters": "--max-loop-iters", "time_scale": "--time-scale",
    "json": "--json", "store": "--store", "stats_file": "--stats-file", "comm_cus": "--comm-cus",
    "comm_lanes": "--comm-lanes", "pp_schedule": "--pp-schedule", "zero": "--zero", "cp_algo": "--cp-algo", "pp_virtual": "--pp-virtual",
    "ranks": "--ranks", "ep_imbalance": "--ep-imbalance", "rccl_max_ctas": "--rccl-max-ctas",
}
_BOOL = {"in_place": "--in-place", "optimizer": "--optimizer", "loop": "--loop", "quiet": "--quiet",
         "silent": "--silent", "graph": "--graph", "trace": "--trace", "ep_overlap": "--ep-overlap",
         "sequence_parallel": "--sequence-parallel"}


def build_args(strategy: str, model: str, *params: int, base_path: str = ".", topology: bool = False,
               **opts: Any) -> List[str]:
    names = POSITIONAL[strategy]
    if len(params) != len(names):
        raise TypeError(f"{strategy} needs {names}, got {params}")
    args = [model] + [str(int(p)) for p in params] + [base_path]
    if not topology:
        args.append("--no-topology")
    for k, v in opts.items():
        if v is None:
            continue
        if k in _BOOL:
            if v:
                args.append(_BOOL[k])
        elif k in _FLAG:
            args += [_FLAG[k], str(v)]
        else:
            raise TypeError(f"unknown option {k!r}")
    return args


def run(strategy: str, model: str, *params: int, **kw: Any) -> Dict[str, Any]:
    return _native.run_raw(strategy, build_args(strategy, model, *params, **kw))
