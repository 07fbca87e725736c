"""Scaling table from bench.py result lines (one JSON line per GPU count).

    python -m dlnetbench_amd bench-report BENCH_N1.json BENCH_N8.json ...
    python -m dlnetbench_amd bench-report runs.jsonl --csv scaling.csv

Every input holds bench.py JSON lines (a file with one line, a JSONL of
several, a JSON array of them, or any JSON document that nests them, e.g. a
driver's scaling record); other lines are skipped, so a captured stdout
works as is. Rows are sorted by ``n_gpus``. Columns: the headline
iteration and its weak-scaling efficiency against the smallest N
(T_min / T_N; the headline keeps per-GPU work fixed), the headline's
all-gather / reduce-scatter bus bandwidth, and the secondary blocks when
present: the comm-bound ViT-H DP step (RCCL, RCCL without the CTA cap,
geometric buckets, our xgmi kernels), the headline FSDP step over xgmi as a
busbw ratio to RCCL, the multi-rank exactness verdict (RCCL / xgmi, the xgmi
release mode that passed) with RCCL's own rank count, and the N = 8 hybrid
configs (C3 hybrid_3d, C4 hybrid_3d_moe) against their GPipe floors.

Reference equivalent: the scaling plots of plots/plot_dp.py:80-145 start
from the per-run DataFrame; this is the same view for the bench contract's
one-line-per-run output.
"""
from __future__ import annotations

import argparse
import json
import sys
from typing import Any, Dict, Iterable, List, Optional


def _walk(obj: Any) -> Iterable[Dict[str, Any]]:
    """Every dict inside a JSON document that looks like a bench.py line
    (a driver's scaling record may nest the per-N lines at any depth)."""
    if isinstance(obj, dict):
        if "metric" in obj and "n_gpus" in obj and "value" in obj:
            yield obj
            return
        for v in obj.values():
            yield from _walk(v)
    elif isinstance(obj, list):
        for v in obj:
            yield from _walk(v)
    elif isinstance(obj, str) and '"metric"' in obj:
        yield from _lines(obj)  # a captured stdout kept as a string


def _lines(text: str) -> Iterable[Dict[str, Any]]:
    text = text.strip()
    if text.startswith("[") or (text.startswith("{") and "\n" not in text.rstrip()):
        try:
            yield from _walk(json.loads(text))
            return
        except json.JSONDecodeError:
            pass
    elif text.startswith("{"):
        try:  # one pretty-printed document
            yield from _walk(json.loads(text))
            return
        except json.JSONDecodeError:
            pass
    for ln in text.splitlines():
        ln = ln.strip()
        if not ln.startswith("{"):
            continue
        try:
            d = json.loads(ln)
        except json.JSONDecodeError:
            continue
        yield from _walk(d)


def load(paths: List[str]) -> List[Dict[str, Any]]:
    """bench.py result lines (dicts with "metric" and "n_gpus") from the inputs, sorted by n_gpus."""
    out = []
    for p in paths:
        with (sys.stdin if p == "-" else open(p)) as f:
            out += [d for d in _lines(f.read()) if "metric" in d and "n_gpus" in d and "value" in d]
    # one run may appear twice in a record (the captured line and a parsed
    # copy of part of it): keep the fullest copy of each
    best: Dict[tuple, Dict[str, Any]] = {}
    for d in out:
        k = (d["n_gpus"], d["value"], d.get("steps"))
        if k not in best or len(d) > len(best[k]):
            best[k] = d
    return sorted(best.values(), key=lambda d: d["n_gpus"])


def _get(d: Optional[dict], *keys: str) -> Any:
    for k in keys:
        if not isinstance(d, dict):
            return None
        d = d.get(k)
    return d


def _largest(by_size: Any) -> Any:
    """busbw at the largest size of a link_bench op ({elements: {...}})."""
    if not isinstance(by_size, dict) or not by_size:
        return None
    k = max(by_size, key=lambda x: int(x))
    return by_size[k].get("busbw_GBps") if isinstance(by_size[k], dict) else None


def rows(lines: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    if not lines:
        return []
    t0 = next((d["ms_per_step"] for d in lines if d.get("ms_per_step")), None)
    out = []
    for d in lines:
        ms = d["ms_per_step"]
        r = {
            "n_gpus": d["n_gpus"],
            "ms_per_step": ms,
            "efficiency": round(t0 / ms, 4) if ms and t0 else None,
            "exposed_comm_ms": d.get("exposed_comm_ms"),
            "ag_busbw_GBps": _get(d, "effective_busbw_GBps", "allgather"),
            "rs_busbw_GBps": _get(d, "effective_busbw_GBps", "reduce_scatter"),
            "c5_ms": _get(d, "comm_bound", "ms_per_step"),
            "c5_busbw_GBps": _get(d, "comm_bound", "allreduce_busbw_GBps"),
            "c5_uncapped_ms": _get(d, "comm_bound", "rccl_default_ctas", "ms_per_step"),
            "c5_geometric_ms": _get(d, "comm_bound", "geometric_buckets", "ms_per_step"),
            "c5_xgmi_ms": _get(d, "comm_bound_xgmi", "ms_per_step"),
            "c5_xgmi_speedup": _get(d, "comm_bound_xgmi", "speedup_vs_comm_bound"),
            "fsdp_xgmi_ag_ratio": _get(d, "headline_xgmi", "busbw_ratio_vs_headline", "allgather"),
            "fsdp_xgmi_rs_ratio": _get(d, "headline_xgmi", "busbw_ratio_vs_headline", "reduce_scatter"),
            "exact_rccl": _get(d, "exact", "rccl"),
            "exact_xgmi": _get(d, "exact", "xgmi"),
            "xgmi_release": _get(d, "exact_detail", "xgmi_release"),
            "rccl_nranks": max((d.get("rccl_nranks") or {}).values(), default=None),
            "c3_ms": _get(d, "hybrid_3d", "ms_per_step"),
            "c3_vs_floor": _get(d, "hybrid_3d", "vs_floor"),
            "c4_ms": _get(d, "hybrid_3d_moe", "ms_per_step"),
            "c4_vs_floor": _get(d, "hybrid_3d_moe", "vs_floor"),
            "c4_overlap_ms": _get(d, "hybrid_3d_moe", "ep_overlap", "ms_per_step"),
            "predicted_ms": d.get("predicted_ms"),
            "fit_eta": _get(d, "model_fit", "eta"),
            "fit_predicted_ms": _get(d, "model_fit", "predicted_ms", "headline"),
            "tl_exposed_max_ms": _get(d, "timeline", "comm_exposed_ms_max"),
            "tl_hidden_frac": _get(d, "timeline", "comm_hidden_frac"),
            "link_ar_busbw_rccl": _largest(_get(d, "link_bench", "rccl", "all_reduce")),
            "link_ar_busbw_xgmi": _largest(_get(d, "link_bench", "xgmi_registered", "all_reduce")),
            "wall_s": _get(d, "phase_seconds", "total"),
            # the backend the headline was timed on (the xgmi fallback when RCCL failed: headline_fallback)
            "backend": _get(d, "config", "backend"),
            "fallback": bool(d.get("headline_fallback")),
        }
        out.append(r)
    return out


def _fmt(v: Any) -> str:
    if v is None:
        return "—"
    if isinstance(v, float):
        return f"{v:.4g}" if abs(v) < 100 else f"{v:.1f}"
    return str(v)


def markdown(rs: List[Dict[str, Any]]) -> str:
    if not rs:
        return "(no bench.py result lines)\n"
    cols = list(rs[0].keys())
    out = ["| " + " | ".join(cols) + " |", "|" + "---:|" * len(cols)]
    out += ["| " + " | ".join(_fmt(r[c]) for c in cols) + " |" for r in rs]
    return "\n".join(out) + "\n"


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("inputs", nargs="+", help="files with bench.py JSON lines ('-' = stdin)")
    ap.add_argument("--csv", default=None, help="also write the table as CSV")
    a = ap.parse_args(argv)
    rs = rows(load(a.inputs))
    sys.stdout.write(markdown(rs))
    if a.csv and rs:
        import csv
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rs[0].keys()))
            w.writeheader()
            w.writerows(rs)
    return 0 if rs else 1


if __name__ == "__main__":
    sys.exit(main())
