"""One command line for the whole toolkit: ``python -m dlnetbench_amd <command> ...``

    run [-n N] [--timeout S] <dp|fsdp|hybrid_2d|hybrid_3d|hybrid_3d_moe|hybrid_cp|hybrid_4d> <args...>
                      launch N ranks of a strategy binary (build/bin/<strategy>)
    commtest [-n N] <args...>
                      exact check / bandwidth sweep of a comm backend (dlnb commtest)
    launch -n N <program ...>   generic N-rank launcher (utils/launch.py)
    sweep | plots | report | plan | schedule-sim | roofline | measure | gemm-bench | clock-check |
    prof-summary | bench-report | download-models | timeline | interference
                      the tools, each with its own --help

The reference spreads these over Makefile targets, SbatchMan jobs and loose
scripts; here every front end is one entry point.
"""
from __future__ import annotations

import importlib
import os
import sys
from typing import List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STRATEGIES = ("dp", "fsdp", "hybrid_2d", "hybrid_3d", "hybrid_3d_moe", "hybrid_cp", "hybrid_4d")

TOOLS = {
    "launch": "dlnetbench_amd.utils.launch",
    "sweep": "dlnetbench_amd.tools.sweep",
    "plots": "dlnetbench_amd.tools.plots",
    "report": "dlnetbench_amd.utils.report",
    "plan": "dlnetbench_amd.parallel.plan",
    "schedule-sim": "dlnetbench_amd.parallel.schedule_sim",
    "roofline": "dlnetbench_amd.models.roofline",
    "measure": "dlnetbench_amd.models.measure",
    "gemm-bench": "dlnetbench_amd.tools.gemm_bench",
    "clock-check": "dlnetbench_amd.tools.clock_check",
    "prof-summary": "dlnetbench_amd.tools.prof_summary",
    "bench-report": "dlnetbench_amd.tools.bench_report",
    "download-models": "dlnetbench_amd.tools.download_models",
    "timeline": "dlnetbench_amd.tools.timeline",
    "interference": "dlnetbench_amd.tools.interference",
}


def _ranks(argv: List[str]):
    """Strip leading -n/--nproc N and --timeout S; returns (n, timeout, rest)."""
    n, timeout, rest = 1, None, list(argv)
    while rest and rest[0] in ("-n", "--nproc", "--timeout"):
        flag = rest.pop(0)
        if not rest:
            raise SystemExit(f"{flag} needs a value")
        val = rest.pop(0)
        if flag == "--timeout":
            timeout = float(val)
        else:
            n = int(val)
    return n, timeout, rest


def _launch(n: int, timeout, cmd: List[str]) -> int:
    if n == 1 and timeout is None:
        import subprocess
        return subprocess.call(cmd)
    from dlnetbench_amd.utils import launch
    code, _ = launch.launch(n, cmd, timeout=timeout)
    return code


def main(argv: Optional[List[str]] = None) -> int:
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0 if argv else 1
    cmd, rest = argv[0], argv[1:]
    bindir = os.path.join(ROOT, "build", "bin")
    if cmd == "run":
        n, timeout, rest = _ranks(rest)
        if not rest or rest[0] not in STRATEGIES:
            print(f"run: expected a strategy ({', '.join(STRATEGIES)})", file=sys.stderr)
            return 1
        return _launch(n, timeout, [os.path.join(bindir, rest[0])] + rest[1:])
    if cmd == "commtest":
        n, timeout, rest = _ranks(rest)
        return _launch(n, timeout, [os.path.join(bindir, "dlnb"), "commtest"] + rest)
    if cmd in TOOLS:
        mod = importlib.import_module(TOOLS[cmd])
        return int(mod.main(rest) or 0)
    print(f"unknown command {cmd!r}; see python -m dlnetbench_amd --help", file=sys.stderr)
    return 1


if __name__ == "__main__":
    raise SystemExit(main())
