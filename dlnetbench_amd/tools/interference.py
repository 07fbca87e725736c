"""Interference benchmark: a victim job alone, then beside an aggressor job.

    python -m dlnetbench_amd interference \\
        --victim "fsdp llama3_8b_16_bfloat16 32 4 . --backend rccl -d 0,1,2,3" --victim-ranks 4 \\
        --aggressor "dp vit_h_32_float8 8 . --backend rccl -d 4,5,6,7" --aggressor-ranks 4 [--json out.json]

The reference builds every driver a second time with -DPROXY_LOOP as a
background traffic generator (the ``*_loop`` binaries, Makefile.common:90-105;
SURVEY.md §2.1 C15) and leaves pairing them with a measured job to the batch
system. This tool does the pairing on one node: it runs the victim to
completion alone, starts the aggressor in ``--loop`` mode (its own ranks,
rendezvous and communicators), waits until it is running, runs the victim
again, stops the aggressor, and reports the victim's iteration time and
per-collective bus bandwidth both ways.

On an MI355X node the two jobs can share GPUs (contention for CUs, HBM and
the hardware queues) or sit on disjoint GPUs (sharing only the xGMI mesh's
links where their rings cross, and the host). The aggressor's launch carries
a hard time limit, so it can never outlive the tool.
"""
from __future__ import annotations

import argparse
import json
import os
import shlex
import signal
import subprocess
import sys
import tempfile
import time
from typing import Any, Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BIN = os.path.join(ROOT, "build", "bin")
STRATEGIES = ("dp", "fsdp", "hybrid_2d", "hybrid_3d", "hybrid_3d_moe", "hybrid_cp", "hybrid_4d")


def _cmd(spec: str) -> List[str]:
    args = shlex.split(spec)
    if not args or args[0] not in STRATEGIES:
        raise ValueError(f"job must start with a strategy ({', '.join(STRATEGIES)}): {spec!r}")
    return [os.path.join(BIN, args[0])] + args[1:]


def _run_victim(cmd: List[str], n: int, timeout: float, env: Dict[str, str]) -> Dict[str, Any]:
    fd, out = tempfile.mkstemp(prefix="dlnb_victim_", suffix=".json")
    os.close(fd)
    try:
        p = subprocess.run([sys.executable, "-m", "dlnetbench_amd.utils.launch", "-n", str(n), "--timeout",
                            str(timeout)] + cmd + ["--quiet", "--json", out], capture_output=True, text=True,
                           timeout=timeout + 30, env=env, cwd=ROOT)
        if p.returncode != 0:
            raise RuntimeError(f"victim exited {p.returncode}: {(p.stderr or '')[-800:]}")
        with open(out) as f:
            return json.load(f)
    finally:
        os.remove(out)


def _summary(doc: Dict[str, Any]) -> Dict[str, Any]:
    it = doc["global"]["dlnb"]["iteration"]
    comm: Dict[str, Any] = {}
    for r in doc["ranks"]:
        for op, c in (r.get("comm") or {}).items():
            e = comm.setdefault(op, {"busbw_GBps": [], "algbw_GBps": []})
            e["busbw_GBps"].append(c.get("busbw_GBps", 0.0))
            e["algbw_GBps"].append(c.get("algbw_GBps", 0.0))
    comm = {op: {k: round(min(v), 3) for k, v in e.items()} for op, e in comm.items()}  # slowest rank
    return {"median_ms": round(it["median_ms"], 4), "mean_ms": round(it["mean_ms"], 4),
            "p95_ms": round(it["p95_ms"], 4), "floor_ms": round(it["compute_floor_ms"], 4),
            "backend": doc["global"].get("backend"), "world_size": doc["global"].get("world_size"), "comm": comm}


def _start_aggressor(cmd: List[str], n: int, limit_s: float, env: Dict[str, str], log) -> subprocess.Popen:
    # --loop: iterations until stopped; the launcher's --timeout is the hard stop
    return subprocess.Popen([sys.executable, "-m", "dlnetbench_amd.utils.launch", "-n", str(n), "--timeout",
                             str(limit_s)] + cmd + ["--loop", "--quiet"], stdout=log, stderr=subprocess.STDOUT,
                            env=env, cwd=ROOT)


def _stop(p: subprocess.Popen) -> Optional[int]:
    """SIGINT makes the launcher terminate its ranks; SIGKILL if it does not exit."""
    if p.poll() is None:
        p.send_signal(signal.SIGINT)
        try:
            p.wait(timeout=30)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait(timeout=10)
    return p.returncode


def run(victim: str, victim_ranks: int, aggressor: str, aggressor_ranks: int, warm_s: float = 3.0,
        timeout: float = 600.0, repeats: int = 1) -> Dict[str, Any]:
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("PYTHONPATH", ROOT)
    vcmd, acmd = _cmd(victim), _cmd(aggressor)
    docs = [_run_victim(vcmd, victim_ranks, timeout, env) for _ in range(repeats)]
    alone = [_summary(d) for d in docs]
    # Fixed-work compute (gemm-work / flops) keeps its alone calibration: a
    # calibration taken beside the aggressor would shrink the work to fit.
    fw = docs[0]["global"]["dlnb"]["compute"].get("fixed_work")
    venv = dict(env)
    if fw:
        venv["DLNB_FIXED_WORK_CAL"] = f"{fw['round_us']!r}:{fw['ktile_us']!r}"
    log = tempfile.TemporaryFile(mode="w+", prefix="dlnb_aggressor_")

    def log_tail() -> str:
        log.flush()
        log.seek(0)
        return log.read()[-800:]

    agg = _start_aggressor(acmd, aggressor_ranks, timeout * repeats + warm_s + 60, env, log)
    try:
        time.sleep(warm_s)
        if agg.poll() is not None:
            raise RuntimeError(f"aggressor exited {agg.returncode} before the victim started: " + log_tail())
        contended = [_summary(_run_victim(vcmd, victim_ranks, timeout, venv)) for _ in range(repeats)]
        running = agg.poll() is None
    finally:
        code = _stop(agg)
        tail = log_tail()
        log.close()
    if not running:
        raise RuntimeError(f"aggressor stopped while the victim ran (exit {code}): {tail}")
    a = min(alone, key=lambda s: s["median_ms"])
    c = max(contended, key=lambda s: s["median_ms"])
    comm = {}
    for op in a["comm"]:
        if op in c["comm"]:
            x, y = a["comm"][op]["busbw_GBps"], c["comm"][op]["busbw_GBps"]
            comm[op] = {"alone_busbw_GBps": x, "contended_busbw_GBps": y,
                        "busbw_ratio": round(y / x, 4) if x else None}
    return {"victim": victim, "victim_ranks": victim_ranks, "aggressor": aggressor + " --loop",
            "aggressor_ranks": aggressor_ranks, "alone": a, "contended": c,
            "slowdown": round(c["median_ms"] / a["median_ms"], 4) if a["median_ms"] else None,
            "comm": comm, "repeats": repeats,
            "fixed_work_cal": venv.get("DLNB_FIXED_WORK_CAL")}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--victim", required=True, help='"<strategy> <positional args> [flags]" (quote it)')
    ap.add_argument("--victim-ranks", type=int, default=1)
    ap.add_argument("--aggressor", required=True, help='"<strategy> <positional args> [flags]", run with --loop')
    ap.add_argument("--aggressor-ranks", type=int, default=1)
    ap.add_argument("--warm-s", type=float, default=3.0, help="aggressor head start before the victim runs")
    ap.add_argument("--timeout", type=float, default=600.0, help="per victim run")
    ap.add_argument("--repeats", type=int, default=1, help="victim runs per phase (best alone, worst contended)")
    ap.add_argument("--json", default=None)
    a = ap.parse_args(argv)
    r = run(a.victim, a.victim_ranks, a.aggressor, a.aggressor_ranks, a.warm_s, a.timeout, a.repeats)
    text = json.dumps(r, indent=1)
    if a.json:
        with open(a.json, "w") as f:
            f.write(text + "\n")
    print(text)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
