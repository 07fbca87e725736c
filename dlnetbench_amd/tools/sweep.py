"""Experiment sweeps with checkpoint/resume.

The reference orchestrates experiments outside the repository with
SbatchMan (.gitignore:18-19, plots/parser.py:221) and sweeps the collective
library's knobs through job variables (plots/plot_dp.py:23-26). This tool
replaces that for a single node: it expands a matrix of
{strategy, model, parallel params, world sizes, options, environment knobs},
runs each point with the dlnb launcher (one process per GPU), and appends one
JSON line per finished point to a results file. Re-running the same sweep
skips points already in the file, so an interrupted sweep resumes where it
stopped (the checkpoint/resume mechanism SURVEY.md §5 calls for).

    python -m dlnetbench_amd.tools.sweep sweep.json --out results.jsonl
    python -m dlnetbench_amd.tools.sweep --quick            # built-in smoke sweep

Sweep file (JSON or YAML):
    {"base_path": ".", "points": [
      {"strategy": "dp", "model": "vit_h_32_float8", "params": [8],
       "world": [1, 2, 4, 8], "opts": {"warmup": 2, "runs": 5},
       "env": {"NCCL_PROTO": ["Simple", "LL128"]}}]}
"params" entries may be the string "W" (replaced by the world size).
"""
from __future__ import annotations

import argparse
import hashlib
import itertools
import json
import os
import sys
import time
from typing import Iterator, List

from ..engine import build_args
from ..utils import launch, report

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

QUICK = {
    "base_path": os.path.join(ROOT, "tests", "data"),
    "points": [
        {"strategy": "dp", "model": "tiny_dense_8_bfloat16", "params": [4], "world": [1, 2],
         "opts": {"warmup": 1, "runs": 2}},
        {"strategy": "fsdp", "model": "tiny_dense_8_bfloat16", "params": [4, "W"], "world": [1, 2],
         "opts": {"warmup": 1, "runs": 2}},
    ],
}


def expand(spec: dict) -> Iterator[dict]:
    for p in spec["points"]:
        worlds = p.get("world", [1])
        env = p.get("env", {})
        env_keys = sorted(env)
        env_vals = [env[k] if isinstance(env[k], list) else [env[k]] for k in env_keys]
        for w in worlds:
            for combo in itertools.product(*env_vals) if env_keys else [()]:
                params = [w if x == "W" else x for x in p.get("params", [])]
                yield {"strategy": p["strategy"], "model": p["model"], "params": params, "world": w,
                       "opts": p.get("opts", {}), "env": dict(zip(env_keys, combo)),
                       "base_path": p.get("base_path", spec.get("base_path", "."))}


def point_key(pt: dict) -> str:
    blob = json.dumps({k: pt[k] for k in ("strategy", "model", "params", "world", "opts", "env")}, sort_keys=True)
    return hashlib.sha1(blob.encode()).hexdigest()[:16]


def done_keys(path: str) -> set:
    keys = set()
    if os.path.exists(path):
        with open(path) as f:
            for line in f:
                try:
                    keys.add(json.loads(line)["key"])
                except (ValueError, KeyError):
                    pass
    return keys


def run_point(pt: dict, binary_dir: str, timeout: float) -> dict:
    args = build_args(pt["strategy"], pt["model"], *pt["params"], base_path=pt["base_path"], quiet=True,
                      **pt["opts"])
    env = dict(os.environ)
    env.update({k: str(v) for k, v in pt["env"].items()})
    t0 = time.time()
    code, outs = launch.launch(pt["world"], [os.path.join(binary_dir, pt["strategy"]), *args], timeout=timeout,
                               capture=True, env=env)
    docs = report.parse_output(outs[0] or "") if outs else {}
    rec = {"key": point_key(pt), "point": pt, "exit_code": code, "wall_s": time.time() - t0}
    if docs:
        doc = next(iter(docs.values()))
        rec["summary"] = report.summary(doc)
        rec["report"] = doc
    else:
        rec["tail"] = "".join(o or "" for o in outs)[-2000:] if outs else ""
    return rec


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("spec", nargs="?", help="sweep file (JSON or YAML)")
    ap.add_argument("--quick", action="store_true", help="run the built-in tiny sweep")
    ap.add_argument("--out", default="sweep_results.jsonl")
    ap.add_argument("--bin", default=os.path.join(ROOT, "build", "bin"))
    ap.add_argument("--timeout", type=float, default=1800)
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    if a.quick:
        spec = QUICK
    elif a.spec:
        with open(a.spec) as f:
            text = f.read()
        try:
            spec = json.loads(text)
        except ValueError:
            import yaml
            spec = yaml.safe_load(text)
    else:
        ap.error("give a sweep file or --quick")
    done = done_keys(a.out)
    pts: List[dict] = list(expand(spec))
    todo = [p for p in pts if point_key(p) not in done]
    print(f"[sweep] {len(pts)} points, {len(pts) - len(todo)} already done, {len(todo)} to run", file=sys.stderr)
    rc = 0
    for pt in todo:
        if a.dry_run:
            print(json.dumps(pt))
            continue
        rec = run_point(pt, a.bin, a.timeout)
        with open(a.out, "a") as f:
            f.write(json.dumps(rec) + "\n")
        s = rec.get("summary", {})
        print(f"[sweep] {pt['strategy']} {pt['model']} W={pt['world']} rc={rec['exit_code']} "
              f"median={s.get('median_ms')} ms", file=sys.stderr)
        rc = rc or rec["exit_code"]
    return rc


if __name__ == "__main__":
    raise SystemExit(main())
