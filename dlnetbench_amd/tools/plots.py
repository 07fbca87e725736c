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
    python -m dlnetbench_amd.tools.plots knobs results.jsonl -o knobs.png [--metric barrier]
    python -m dlnetbench_amd.tools.plots knobs-pareto results.jsonl -o knobs_pareto.png
    python -m dlnetbench_amd.tools.plots timeline trace.json -o timeline.png [--iter N]

Collective-library knobs (the reference's PROTOCOL x ALGO and THREADS x
CHANNELS axes, plot_dp.py:23-26) are read from each sweep point's
environment: NCCL_PROTO, NCCL_ALGO, NCCL_NTHREADS and NCCL_MIN_NCHANNELS /
NCCL_MAX_NCHANNELS for RCCL, DLNB_XGMI_BLOCKS for the xgmi kernels (their
"channels"); a knob a point does not set shows as "default".
"""
from __future__ import annotations

import argparse
import itertools
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


# ---------------------------------------------------------------- style maps
# (py_utils.py:8-13, :123-132)

MARKERS = ["o", "s", "^", "d", "v", "P", "*", "X", ">", "<", "h", "p"]
LINESTYLES = ["-", ":", "-.", "--"]
COLORS = ["#1f77b4", "#ff7f0e", "#2ca02c", "#d62728", "#9467bd", "#8c564b", "#e377c2", "#7f7f7f", "#bcbd22",
          "#17becf"]


def create_color_map(values: Sequence) -> Dict:
    """One colour per value, cycling through a 10-colour palette."""
    return {v: c for v, c in zip(values, itertools.cycle(COLORS))}


def create_marker_map(values: Sequence) -> Dict:
    return {v: m for v, m in zip(values, itertools.cycle(MARKERS))}


def create_linestyle_map(values: Sequence) -> Dict:
    return {v: ls for v, ls in zip(values, itertools.cycle(LINESTYLES))}


def add_zoom_inset(ax, zoom_region: Tuple[float, float, float, float],
                   inset_position: Tuple[float, float, float, float] = (0.6, 0.6, 0.35, 0.35),
                   draw_rect: bool = True):
    """Magnified copy of the lines and scatter points of `ax` inside zoom_region
    = (x1, x2, y1, y2), drawn at inset_position (axes fractions x0, y0, w, h),
    with a dashed rectangle marking the region on the main axes
    (py_utils.add_zoom_inset). Returns the inset axes."""
    from matplotlib.patches import Rectangle
    x1, x2, y1, y2 = zoom_region
    axins = ax.inset_axes(list(inset_position))
    for line in ax.get_lines():
        axins.plot(line.get_xdata(), line.get_ydata(), color=line.get_color(), linestyle=line.get_linestyle(),
                   linewidth=line.get_linewidth(), marker=line.get_marker(), markersize=line.get_markersize(),
                   alpha=line.get_alpha())
    for coll in ax.collections:
        offs = coll.get_offsets()
        if len(offs):
            axins.scatter(offs[:, 0], offs[:, 1], c=coll.get_facecolors(), s=coll.get_sizes(),
                          marker=(coll.get_paths()[0] if coll.get_paths() else "o"))
    axins.set_xlim(x1, x2)
    axins.set_ylim(y1, y2)
    axins.tick_params(labelsize=6)
    axins.grid(alpha=0.3)
    if draw_rect:
        ax.add_patch(Rectangle((x1, y1), x2 - x1, y2 - y1, fill=False, edgecolor="black", linestyle="dashed",
                               linewidth=1))
    return axins


# ---------------------------------------------------------------- knobs

def knobs(rec: dict) -> Dict[str, str]:
    """Collective-library knobs of one sweep record (see the module doc)."""
    env = {k: str(v) for k, v in rec.get("point", {}).get("env", {}).items()}
    ch = env.get("NCCL_MAX_NCHANNELS") or env.get("NCCL_MIN_NCHANNELS") or env.get("DLNB_XGMI_BLOCKS")
    return {"protocol": env.get("NCCL_PROTO", "default"), "algorithm": env.get("NCCL_ALGO", "default"),
            "threads": env.get("NCCL_NTHREADS", "default"), "channels": ch or "default"}


def _knob_sort_key(v: str):
    return (0, float(v), "") if re.fullmatch(r"[0-9.]+", v) else (1, 0.0, v)


def knob_table(recs: List[dict], metric: str = "runtime") -> List[dict]:
    """One row per record: model, world size, knobs, and the metric in ms
    (runtime = median iteration; barrier = mean exposed all-reduce wait)."""
    rows = []
    for r in recs:
        rep = r["report"]
        g = rep["global"]
        if metric == "barrier":
            vals = [b * 1e3 for rk in rep["ranks"] for b in rk.get("barrier_time", [])]
            if not vals:
                continue
            y = sum(vals) / len(vals)
        else:
            y = g["dlnb"]["iteration"]["median_ms"]
        e = [x for rk in rep["ranks"] for x in rk.get("energy_consumed", [])]
        runs = max(1, len(rep["ranks"][0].get("energy_consumed", []))) if e else 1
        rows.append(dict(knobs(r), model=g.get("model_name"), world=g.get("world_size"), value_ms=y,
                         energy_J=(sum(e) / runs) if e else None,
                         msg_bytes=g.get("msg_size_avg_bytes") or g.get("allgather_msg_size_bytes")))
    return rows


def plot_knobs(recs: List[dict], out: str, metric: str = "runtime") -> Dict[Tuple[str, str], int]:
    """Protocol x algorithm facets (rows x columns); inside each facet the
    metric against world size, one line per threads x channels combination
    (plot_dp.py:23-26 knob grid). Returns {(protocol, algorithm): points}."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    rows = knob_table(recs, metric)
    protos = sorted({r["protocol"] for r in rows}, key=_knob_sort_key) or ["default"]
    algos = sorted({r["algorithm"] for r in rows}, key=_knob_sort_key) or ["default"]
    tcs = sorted({(r["threads"], r["channels"]) for r in rows},
                 key=lambda t: (_knob_sort_key(t[0]), _knob_sort_key(t[1])))
    colors, marks = create_color_map(tcs), create_marker_map(tcs)
    fig, axes = plt.subplots(len(protos), len(algos), figsize=(4.2 * len(algos), 3.4 * len(protos)), squeeze=False,
                             sharex=True, sharey=True)
    counts: Dict[Tuple[str, str], int] = {}
    for i, pr in enumerate(protos):
        for j, al in enumerate(algos):
            ax = axes[i][j]
            sub = [r for r in rows if r["protocol"] == pr and r["algorithm"] == al]
            counts[(pr, al)] = len(sub)
            for tc in tcs:
                pts = sorted((r["world"], r["value_ms"]) for r in sub if (r["threads"], r["channels"]) == tc)
                if pts:
                    ax.plot([p[0] for p in pts], [p[1] for p in pts], marker=marks[tc], color=colors[tc],
                            label=f"T{tc[0]} x C{tc[1]}")
            ax.set_title(f"{pr} x {al}", fontsize=9)
            ax.set_xscale("log", base=2)
            ax.grid(alpha=0.3)
            if i == len(protos) - 1:
                ax.set_xlabel("GPUs")
            if j == 0:
                ax.set_ylabel("barrier time (ms)" if metric == "barrier" else "iteration (ms)")
    handles, labels = axes[0][0].get_legend_handles_labels()
    for ax in axes.flat:
        h, l = ax.get_legend_handles_labels()
        for hh, ll in zip(h, l):
            if ll not in labels:
                handles.append(hh)
                labels.append(ll)
    if handles:
        fig.legend(handles, labels, loc="center right", fontsize=7, title="threads x channels")
    fig.tight_layout(rect=(0, 0, 0.85, 1))
    fig.savefig(out, dpi=150)
    plt.close(fig)
    return counts


def pareto_staircase(points: Sequence[Tuple[float, float]]) -> List[Tuple[float, float]]:
    """Vertices of the staircase through the Pareto front (minimise both),
    sorted by x (plots_pareto_energy.py draw_pareto_frontier)."""
    fr = sorted(points[i] for i in pareto_front(points))
    out: List[Tuple[float, float]] = []
    for k, (x, y) in enumerate(fr):
        if k:
            out.append((x, fr[k - 1][1]))
        out.append((x, y))
    return out


def plot_knobs_pareto(recs: List[dict], out: str) -> Dict[str, int]:
    """Energy vs runtime per model (one subplot each): colour = protocol x
    algorithm, marker = threads x channels, staircase Pareto frontier
    (plots_pareto_energy.py:107-234). Returns {model: points}."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from matplotlib.lines import Line2D
    rows = [r for r in knob_table(recs) if r["energy_J"] is not None]
    models = sorted({r["model"] for r in rows}) or ["(no energy data)"]
    pa = sorted({f"{r['protocol']} x {r['algorithm']}" for r in rows})
    tc = sorted({f"T{r['threads']} x C{r['channels']}" for r in rows})
    colors, marks = create_color_map(pa), create_marker_map(tc)
    fig, axes = plt.subplots(1, len(models), figsize=(6.5 * len(models), 5), squeeze=False)
    counts: Dict[str, int] = {}
    for ax, m in zip(axes[0], models):
        sub = [r for r in rows if r["model"] == m]
        counts[m] = len(sub)
        for r in sub:
            ax.scatter(r["energy_J"], r["value_ms"], color=colors[f"{r['protocol']} x {r['algorithm']}"],
                       marker=marks[f"T{r['threads']} x C{r['channels']}"], s=70, edgecolor="black", linewidth=0.6,
                       alpha=0.8, zorder=5)
        stair = pareto_staircase([(r["energy_J"], r["value_ms"]) for r in sub])
        if len(stair) > 1:
            ax.plot([p[0] for p in stair], [p[1] for p in stair], color="red", lw=2, zorder=10)
        msg = sub[0]["msg_bytes"] if sub else None
        ax.set_title(f"{m}" + (f" (message {format_bytes(msg)})" if msg else ""), fontsize=10)
        ax.set_xlabel("energy per iteration, all ranks (J)")
        ax.set_ylabel("iteration time (ms)")
        ax.grid(alpha=0.3)
    items = [Line2D([0], [0], color="red", lw=2, label="Pareto frontier")]
    items += [Line2D([0], [0], marker="o", color="w", markerfacecolor=colors[p], markeredgecolor="black",
                     label=p) for p in pa]
    items += [Line2D([0], [0], marker=marks[t], color="w", markerfacecolor="gray", markeredgecolor="black",
                     label=t) for t in tc]
    fig.legend(handles=items, loc="center right", fontsize=7)
    fig.tight_layout(rect=(0, 0, 0.82, 1))
    fig.savefig(out, dpi=150)
    plt.close(fig)
    return counts


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


def plot_timeline(trace: str, out: str, iteration=None) -> Dict[str, int]:
    """Gantt chart of a --timeline trace (csrc/src/timeline.cpp): one row per
    (rank, stream), compute spans in grey, collectives coloured by operation,
    one iteration (the last one by default). Returns spans drawn per category."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    with open(trace) as f:
        doc = json.load(f)
    ev = [e for e in doc["traceEvents"] if e.get("ph") == "X"]
    names = {(m["pid"], m["tid"]): m["args"]["name"] for m in doc["traceEvents"]
             if m.get("ph") == "M" and m.get("name") == "thread_name"}
    if iteration is None:
        iteration = max((e["args"]["iter"] for e in ev), default=0)
    ev = [e for e in ev if e["args"]["iter"] == iteration]
    rows = sorted({(e["pid"], e["tid"]) for e in ev})
    t0 = min((e["ts"] for e in ev), default=0.0)
    ops = sorted({e["name"].split(" ")[0] for e in ev if e["cat"] != "compute"})
    colors = create_color_map(ops)
    fig, ax = plt.subplots(figsize=(12, 0.4 * len(rows) + 1.5))
    drawn: Dict[str, int] = {}
    for e in ev:
        y = rows.index((e["pid"], e["tid"]))
        op = e["name"].split(" ")[0]
        c = "0.75" if e["cat"] == "compute" else colors[op]
        ax.barh(y, e["dur"] / 1e3, left=(e["ts"] - t0) / 1e3, color=c, edgecolor="none", height=0.8)
        drawn[e["cat"]] = drawn.get(e["cat"], 0) + 1
    ax.set_yticks(range(len(rows)))
    ax.set_yticklabels([f"r{p} {names.get((p, t), t)}" for p, t in rows], fontsize=7)
    ax.invert_yaxis()
    ax.set_xlabel("ms")
    ax.set_title(f"{doc.get('otherData', {}).get('strategy', '')} iteration {iteration}")
    import matplotlib.patches as mpatches
    handles = [mpatches.Patch(color="0.75", label="compute")] + [mpatches.Patch(color=colors[o], label=o) for o in ops]
    ax.legend(handles=handles, fontsize=7, loc="upper right")
    fig.tight_layout()
    fig.savefig(out, dpi=150)
    plt.close(fig)
    return drawn


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("kind", choices=["scaling", "barrier", "pareto", "knobs", "knobs-pareto", "timeline"])
    ap.add_argument("inputs", nargs="+")
    ap.add_argument("-o", "--out", default="plot.png")
    ap.add_argument("--metric", choices=["runtime", "barrier"], default="runtime", help="knobs: y axis")
    ap.add_argument("--iter", type=int, default=None, help="timeline: iteration (default: the last)")
    a = ap.parse_args(argv)
    if a.kind == "timeline":
        plot_timeline(a.inputs[0], a.out, a.iter)
        print(a.out)
        return 0
    recs = [r for p in a.inputs for r in load_records(p)]
    if a.kind == "knobs":
        plot_knobs(recs, a.out, a.metric)
    else:
        {"scaling": plot_scaling, "barrier": plot_barrier, "pareto": plot_pareto,
         "knobs-pareto": plot_knobs_pareto}[a.kind](recs, a.out)
    print(a.out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
