"""Python front-end for the native benchmark runtime.

``run("fsdp", "llama3_8b_16_bfloat16", 32, 8, base_path=".", warmup=1, runs=3)``
runs one rank of a benchmark in this process (rank identity comes from the
environment exactly like the CLI binaries) and returns the report document:
``{"section", "title", "global": {...}, "ranks": [{...}, ...]}`` with the
reference's key names plus ``global["dlnb"]`` extras.
"""
from __future__ import annotations

import json
import os
import subprocess
import tempfile
from typing import Any, Dict, List, Optional

from . import _native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

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
    "dp_buckets": "--dp-buckets", "dp_bucket_ratio": "--dp-bucket-ratio", "max_loop_iters": "--max-loop-iters", "time_scale": "--time-scale",
    "json": "--json", "store": "--store", "stats_file": "--stats-file", "comm_cus": "--comm-cus",
    "comm_lanes": "--comm-lanes", "pp_schedule": "--pp-schedule", "zero": "--zero", "cp_algo": "--cp-algo", "pp_virtual": "--pp-virtual",
    "ranks": "--ranks", "ep_imbalance": "--ep-imbalance", "rccl_max_ctas": "--rccl-max-ctas",
    "timeline": "--timeline", "timeline_iters": "--timeline-iters",
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


def run_native(strategy: str, model: str, *params: int, timeout: float = 600, env: Optional[Dict[str, str]] = None,
               **kw: Any) -> Dict[str, Any]:
    """Run one rank of a benchmark in a child process of the native binary
    (build/bin/<strategy>) and return its report document.

    The binary never imports torch, so it binds /opt/rocm's HIP runtime and
    RCCL - the stack bench.py measures - even when this process has torch
    (and with it torch's bundled HIP / RCCL) loaded. Raises NativeError with
    the tail of the child's stderr if it fails."""
    binary = os.path.join(ROOT, "build", "bin", strategy)
    if not os.path.exists(binary):
        raise _native.NativeError(f"{binary} is missing: build it with `make`")
    fd, out = tempfile.mkstemp(prefix="dlnb_report_", suffix=".json")
    os.close(fd)
    try:
        kw.setdefault("silent", True)
        args = build_args(strategy, model, *params, json=out, **kw)
        e = dict(os.environ, DLNB_NO_TORCH="1")
        e.update(env or {})
        p = subprocess.run([binary, *args], capture_output=True, text=True, timeout=timeout, env=e)
        if p.returncode != 0:
            raise _native.NativeError(f"{strategy} exited {p.returncode}: {(p.stderr or '')[-1500:]}")
        with open(out) as f:
            return json.load(f)
    finally:
        if os.path.exists(out):
            os.remove(out)
