"""Fold rocprofv3 output into a benchmark report: ``global.dlnb.counters``.

The reference reports host wall-clock timers only (cpp/data_parallel/dp.cpp:
258-264); SURVEY.md §5 asks for rocprof counters in the report. This tool
reads a rocprofv3 kernel trace (``--kernel-trace``, ``*kernel_trace.csv``)
and/or a counter collection (``--pmc``, ``*counter_collection.csv``) of the
same command, groups kernels into classes and writes, per class: calls,
kernel time, and — when the counters were collected — MFMA busy fraction,
MFMA TFLOP/s, and the bytes read / written beyond the L2 (TCC <-> data
fabric: Infinity Cache or HBM; FETCH_SIZE / WRITE_SIZE) with their rate.

    rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof -- python3 bench.py --json r.json ...
    rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv \\
        -d gpurun_out/pmc -- python3 bench.py ...
    python -m dlnetbench_amd.tools.prof_merge r.json gpurun_out/prof gpurun_out/pmc -o r_counters.json

Counter units (rocprofv3 derived metrics): FETCH_SIZE / WRITE_SIZE are KiB;
MFMA MOPS count 512 FLOPs each; MFMA busy is normalised by clock x kernel
time x CUs x 4 SIMDs (MI355X: 256 CUs).

Clock: GRBM_GUI_ACTIVE counts GPU-busy cycles (x 8 XCDs) over the counter
collection window of a dispatch, which is longer than the kernel's own start
/ end stamps by a fixed setup cost - dividing by the kernel time read 2.9-3.5
GHz for 10-us copy / stamp kernels. The clock is therefore derived only from
dispatches of at least LONG_DISPATCH_MS (per class when it has some, else
from every long dispatch of the job, ``clock_source: job``), and a derived
clock above MAX_CLOCK_GHZ (the MI355X peak is 2.4 GHz) or an MFMA busy
fraction above 1 raises instead of being reported.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os
import re
from typing import Dict, Iterable, List, Optional

CUS = 256
XCDS = 8
SIMDS = 4
LONG_DISPATCH_MS = 0.5
MAX_CLOCK_GHZ = 2.5

# first match wins
CLASSES = [
    ("compute_gemm", re.compile(r"gemm", re.I)),
    ("compute_wait", re.compile(r"idle_wait|busy_spin|spin_kernel|sleep", re.I)),
    ("rccl", re.compile(r"nccl|rccl(?!r)", re.I)),
    ("xgmi", re.compile(r"xgmi::|ag_kernel|rs_kernel|ar1_kernel|ar2_kernel|a2a_kernel|send_kernel|recv_kernel|"
                        r"local_reduce|local_coll", re.I)),
    ("copy", re.compile(r"copyBuffer|fillBuffer|memcpy|memset|fill_kernel", re.I)),
    ("timing", re.compile(r"stamp", re.I)),
]


def classify(name: str) -> str:
    for cls, rx in CLASSES:
        if rx.search(name):
            return cls
    return "other"


def _csvs(dirs: Iterable[str], suffix: str) -> List[str]:
    out: List[str] = []
    for d in dirs:
        if os.path.isfile(d) and d.endswith(suffix):
            out.append(d)
        else:
            out += sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))
    return out


def _f(v: Optional[str]) -> float:
    try:
        return float(v) if v not in (None, "") else 0.0
    except ValueError:
        return 0.0


def collect(dirs: List[str]) -> Dict[str, dict]:
    """{class: {calls, time_ms, counters{name: sum}, counter_ms{name: dispatch ms}, kernels{short: calls}}}.

    Counters may come from several --pmc passes (one pass cannot hold every
    counter): each counter keeps the dispatch time of the passes it was
    collected in, so rates derived from it are per pass, never diluted."""
    cls: Dict[str, dict] = collections.defaultdict(
        lambda: {"calls": 0, "time_ms": 0.0, "counters": collections.defaultdict(float),
                 "counter_ms": collections.defaultdict(float), "kernels": collections.Counter(),
                 "gui": []})  # (dispatch ms, GRBM_GUI_ACTIVE) per dispatch
    traced = set()
    for path in _csvs(dirs, "kernel_trace.csv"):
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name", "")
            c = cls[classify(name)]
            c["calls"] += 1
            c["time_ms"] += (_f(r.get("End_Timestamp")) - _f(r.get("Start_Timestamp"))) / 1e6
            c["kernels"][_short(name)] += 1
            traced.add(classify(name))
    for path in _csvs(dirs, "counter_collection.csv"):
        seen = set()
        file_ms: Dict[str, float] = collections.defaultdict(float)
        file_names: Dict[str, set] = collections.defaultdict(set)
        for r in csv.DictReader(open(path)):
            name = r.get("Kernel_Name", "")
            k = classify(name)
            c = cls[k]
            c["counters"][r["Counter_Name"]] += _f(r.get("Counter_Value"))
            file_names[k].add(r["Counter_Name"])
            key = (r.get("Dispatch_Id"), r.get("Agent_Id"))
            ms = (_f(r.get("End_Timestamp")) - _f(r.get("Start_Timestamp"))) / 1e6
            if r["Counter_Name"] == "GRBM_GUI_ACTIVE":
                c["gui"].append((ms, _f(r.get("Counter_Value"))))
            if key not in seen:
                seen.add(key)
                file_ms[k] += ms
                if k not in traced:  # counters without a trace: count the dispatches here
                    c["calls"] += 1
                    c["time_ms"] += ms
                    c["kernels"][_short(name)] += 1
        for k, names in file_names.items():
            for n in names:
                cls[k]["counter_ms"][n] += file_ms[k]
    return cls


def _short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:80]


def long_dispatch_clock(gui: List[tuple]) -> Optional[float]:
    """Clock (Hz) from the dispatches of at least LONG_DISPATCH_MS:
    sum(GRBM_GUI_ACTIVE) / XCDs over their summed kernel time; None if none."""
    long = [(ms, g) for ms, g in gui if ms >= LONG_DISPATCH_MS and g > 0]
    if not long:
        return None
    hz = sum(g for _, g in long) / XCDS / (sum(ms for ms, _ in long) * 1e-3)
    if hz / 1e9 > MAX_CLOCK_GHZ:
        raise ValueError(f"derived clock {hz / 1e9:.3f} GHz > {MAX_CLOCK_GHZ} GHz from {len(long)} dispatches "
                         f">= {LONG_DISPATCH_MS} ms: GRBM_GUI_ACTIVE or the timestamps are not what prof_merge assumes")
    return hz


def derive(c: dict, job_clock: Optional[float] = None) -> dict:
    """Per-class summary with derived rates (only those whose counters exist)."""
    k = c["counters"]
    out = {"calls": c["calls"], "time_ms": round(c["time_ms"], 4),
           "kernels": dict(c["kernels"].most_common(6))}

    def rate(name: str) -> float:  # counter per second over the passes that collected it
        ms = c["counter_ms"].get(name, 0.0)
        return k.get(name, 0.0) / (ms * 1e-3) if ms > 0 else 0.0

    hz = long_dispatch_clock(c.get("gui", []))
    source = "class"
    if hz is None and job_clock and c.get("gui"):
        hz, source = job_clock, "job"
    if hz:
        out["clock_GHz"] = round(hz / 1e9, 3)
        out["clock_source"] = source
        if "SQ_VALU_MFMA_BUSY_CYCLES" in k:
            busy = rate("SQ_VALU_MFMA_BUSY_CYCLES") / (hz * CUS * SIMDS)
            if busy > 1.0 + 1e-6:
                raise ValueError(f"MFMA busy fraction {busy:.3f} > 1 (clock {hz / 1e9:.3f} GHz)")
            out["mfma_busy"] = round(busy, 4)
    mops = sum(rate(n) for n in k if n.startswith("SQ_INSTS_VALU_MFMA_MOPS"))
    if mops:
        out["mfma_TFLOPs"] = round(mops * 512 / 1e12, 1)
    if "FETCH_SIZE" in k or "WRITE_SIZE" in k:  # L2 misses / write-backs to the fabric (MALL or HBM)
        out["fabric_read_bytes"] = k.get("FETCH_SIZE", 0.0) * 1024
        out["fabric_write_bytes"] = k.get("WRITE_SIZE", 0.0) * 1024
        out["fabric_GBps"] = round((rate("FETCH_SIZE") + rate("WRITE_SIZE")) * 1024 / 1e9, 1)
    if k:
        out["counters"] = dict(k)
    return out


def merge(report: dict, dirs: List[str]) -> dict:
    cls = collect(dirs)
    job_clock = long_dispatch_clock([d for c in cls.values() for d in c["gui"]])
    classes = {name: derive(c, job_clock) for name, c in sorted(cls.items())}
    total = sum(v["time_ms"] for v in classes.values())
    for v in classes.values():
        v["time_pct"] = round(100.0 * v["time_ms"] / total, 2) if total else 0.0
    # The deadline GEMM runs on `deadline_grid` CUs (the rest are left to the
    # collectives): its MFMA busy fraction on the CUs it occupies.
    grid = report.get("global", {}).get("dlnb", {}).get("compute", {}).get("deadline_grid")
    cg = classes.get("compute_gemm")
    if grid and cg and "mfma_busy" in cg:
        cg["grid_cus"] = grid
        cg["mfma_busy_on_grid"] = round(cg["mfma_busy"] * CUS / grid, 4)
    g = report.setdefault("global", {}).setdefault("dlnb", {})
    g["counters"] = {"source": [os.path.basename(os.path.normpath(d)) for d in dirs], "total_kernel_ms": round(total, 4),
                     "classes": classes}
    return report


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("report", help="report JSON (--json of a run / bench.py --json); '-' for an empty one")
    ap.add_argument("prof_dirs", nargs="+", help="rocprofv3 output directories (or CSV files)")
    ap.add_argument("-o", "--out", default=None, help="output JSON (default: overwrite the report)")
    a = ap.parse_args(argv)
    rep = {} if a.report == "-" else json.load(open(a.report))
    merge(rep, a.prof_dirs)
    out = a.out or a.report
    if out == "-":
        print(json.dumps(rep, indent=1))
    else:
        with open(out, "w") as f:
            json.dump(rep, f, indent=1)
        print(out)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
