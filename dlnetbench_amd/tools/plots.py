"""Plots of benchmark results (matplotlib, offline).

Reference equivalents: plots/plot_dp.py (runtime vs world size and
barrier-time scatter per bucket count, sweeping NCCL protocol / algorithm /
threads / channels, :23-163), plots/plots_pareto_energy.py (energy vs
runtime Pareto frontier, :36-234) and plots/py_utils.py (byte formatting,
colour/marker maps, zoom insets, :15-209). Inputs here are sweep JSONL files
(tools/sweep.py) or report JSON files.

    python -m dlnetbench_amd.tools.plots scaling results.jsonl -o scaling.png
    python -m dlnetbench_amd.tools.plots barrier results.jsonl -o barrier.png
    python -m dlnetbench_amd.tools.plots pareto results.jsonl -o pareto.png
"""
from __future__ import annotations

import argparse
import json
import re
from typing import Dict, List, Sequence, Tuple

_UNITS = ["B", "KiB", "MiB", "GiB", "TiB"]


def format_bytes(n: float) -> str:
    """1536 -> '1.5 KiB' (py_utils.format_bytes)."""
    n = float(n)
    for u in _UNITS:
        if abs(n) < 1024 or u == _UNITS[-1]:
            return f"{n:.0f} {u}" if u == "B" else f"{n:.1f} {u}"
        n /= 1024
    return f"{n:.1f} TiB"


def parse_bytes(s: str) -> int:
    """'1.5 KiB' / '2GB' / '512' -> bytes (py_utils.parse_bytes)."""
    m = re.fullmatch(r"\s*([0-9.]+)\s*([KMGT]?i?B?)\s*", s, re.I)
    if not m:
        raise ValueError(f"cannot parse size {s!r}")
    v, u = float(m.group(1)), m.group(2).upper()
    mult = {"": 1, "B": 1, "K": 1e3, "KB": 1e3, "KIB": 1024, "M": 1e6, "MB": 1e6, "MIB": 1024 ** 2,
            "G": 1e9, "GB": 1e9, "GIB": 1024 ** 3, "T": 1e12, "TB": 1e12, "TIB": 1024 ** 4}[u]
    return int(v * mult)


def pareto_front(points: Sequence[Tuple[float, float]]) -> List[int]:
    """Indices of the points not dominated in (minimise x, minimise y)."""
    idx = sorted(range(len(points)), key=lambda i: (points[i][0], points[i][1]))
    front, best_y = [], float("inf")
    for i in idx:
        if points[i][1] < best_y:
            front.append(i)
            best_y = points[i][1]
    return front


def load_records(path: str) -> List[dict]:
    recs = []
    with open(path) as f:
        text = f.read()
    try:
        d = json.loads(text)
        return [{"report": d, "point": {}}]
    except ValueError:
        pass
    for line in text.splitlines():
        if line.strip():
            recs.append(json.loads(line))
    return [r for r in recs if "report" in r]


def _series_label(rec: dict) -> str:
    env = rec.get("point", {}).get("env", {})
    g = rec["report"]["global"]
    lab = f"{g.get('model_name')} {rec['report']['section']}"
    if env:
        lab += " " + ",".join(f"{k}={v}" for k, v in sorted(env.items()))
    return lab


def plot_scaling(recs: List[dict], out: str) -> None:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    series: Dict[str, List[Tuple[int, float]]] = {}
    for r in recs:
        g = r["report"]["global"]
        series.setdefault(_series_label(r), []).append((g["world_size"], g["dlnb"]["iteration"]["median_ms"]))
    fig, ax = plt.subplots(figsize=(7, 4.5))
    for lab, pts in sorted(series.items()):
        pts.sort()
        ax.plot([p[0] for p in pts], [p[1] for p in pts], marker="o", label=lab)
    ax.set_xlabel("GPUs (MI355X)")
    ax.set_ylabel("iteration time (ms, median of max-over-ranks)")
    ax.set_xscale("log", base=2)
    ax.grid(alpha=0.3)
    ax.legend(fontsize=7)
    fig.tight_layout()
    fig.savefig(out, dpi=150)


def plot_barrier(recs: List[dict], out: str) -> None:
    """Exposed communication per bucket count (plot_dp.py barrier scatter)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, ax = plt.subplots(figsize=(7, 4.5))
    for r in recs:
        rep = r["report"]
        if rep["section"] != "dp":
            continue
        nb = rep["global"]["num_buckets"]
        ys = [b * 1e3 for rk in rep["ranks"] for b in rk["barrier_time"]]
        ax.scatter([nb] * len(ys), ys, s=8, alpha=0.6, label=f"W={rep['global']['world_size']}")
    ax.set_xlabel("number of gradient buckets")
    ax.set_ylabel("exposed all-reduce (barrier) time, ms")
    ax.grid(alpha=0.3)
    fig.tight_layout()
    fig.savefig(out, dpi=150)


def plot_pareto(recs: List[dict], out: str) -> None:
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    pts, labels = [], []
    for r in recs:
        rep = r["report"]
        e = [x for rk in rep["ranks"] for x in rk.get("energy_consumed", [])]
        if not e:
            continue
        runs = max(1, len(rep["ranks"][0].get("energy_consumed", [])))
        pts.append((rep["global"]["dlnb"]["iteration"]["median_ms"], sum(e) / runs))
        labels.append(_series_label(r))
    fig, ax = plt.subplots(figsize=(7, 4.5))
    if pts:
        ax.scatter([p[0] for p in pts], [p[1] for p in pts], s=14)
        fr = pareto_front(pts)
        fr_pts = sorted(pts[i] for i in fr)
        ax.plot([p[0] for p in fr_pts], [p[1] for p in fr_pts], "r--", label="Pareto front")
    ax.set_xlabel("iteration time (ms)")
    ax.set_ylabel("energy per iteration, all ranks (J)")
    ax.grid(alpha=0.3)
    if pts:
        ax.legend()
    fig.tight_layout()
    fig.savefig(out, dpi=150)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["scaling", "barrier", "pareto"])
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("-o", "--out", default="plot.png")
    a = ap.parse_args(argv)
    recs = [r for p in a.inputs for r in load_records(p)]
    {"scaling": plot_scaling, "barrier": plot_barrier, "pareto": plot_pareto}[a.kind](recs, a.out)
    print(a.out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
