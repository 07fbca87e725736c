#!/usr/bin/env python3
"""Summaries of rocprofv3 CSV traces (round 5 probes, scripts/probes/lanes_r5.sh).

  trace_queues.py queues <kernel_trace.csv>
      which hardware queues each kind of kernel ran on (compute = the deadline / one-shot GEMMs and idle / spin
      kernels, collective = RCCL / copy / xgmi kernels, gate / stamp / handshake one-wave kernels): lane graphs
      should put every compute dispatch on one queue and every collective on another.
  trace_queues.py api <hip_api_trace.csv> [<kernel_trace.csv>]
      the HIP API calls of the timed loop: per hipGraphLaunch its duration, the slowest calls overall, and the
      calls longer than 100 us with the replay they fell in (the slow replay every 16).
"""
from __future__ import annotations

import csv
import sys
from collections import Counter, defaultdict


def _rows(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def kind(name: str) -> str:
    n = name.lower()
    if "gemm" in n or "idle_wait" in n or "busy_spin" in n:
        return "compute"
    if any(k in n for k in ("nccl", "rccl", "copybuffer", "xgmi", "allreduce", "allgather", "reducescatter")):
        return "collective"
    if any(k in n for k in ("gate_", "stamp_kernel", "host_wait", "host_signal", "set_word")):
        return "sync"
    return "other"


def queues(path: str) -> None:
    rows = _rows(path)
    # the iterations only: from the first compute kernel on (setup's fills and copies run on other queues)
    first = min((int(r["Start_Timestamp"]) for r in rows if kind(r.get("Kernel_Name", "")) == "compute"), default=0)
    rows = [r for r in rows if int(r["Start_Timestamp"]) >= first]
    by = defaultdict(Counter)
    names = defaultdict(Counter)
    for r in rows:
        k = kind(r.get("Kernel_Name", ""))
        q = r.get("Queue_Id", "?")
        by[k][q] += 1
        names[k][r.get("Kernel_Name", "")[:60]] += 1
    for k in ("compute", "collective", "sync", "other"):
        if k in by:
            print(f"{k:10s} queues {dict(by[k])}  kernels {dict(names[k].most_common(3))}")
    comp, coll = set(by.get("compute", {})), set(by.get("collective", {}))
    print(f"compute on {len(comp)} queue(s), collectives on {len(coll)} queue(s), shared: {sorted(comp & coll)}")


def api(path: str, kpath: str | None = None) -> None:
    rows = _rows(path)
    calls = [(r["Function"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    calls.sort(key=lambda c: c[1])
    launches = [c for c in calls if c[0] == "hipGraphLaunch"]
    print(f"{len(calls)} HIP API calls, {len(launches)} hipGraphLaunch")
    for i, (_, a, b) in enumerate(launches):
        print(f"  launch {i:3d} at {(a - launches[0][1]) / 1e6:10.3f} ms: {(b - a) / 1e3:8.1f} us")
    slow = sorted(calls, key=lambda c: c[1] - c[2])[:25]
    print("slowest calls:")
    t0 = calls[0][1] if calls else 0
    for f, a, b in slow:
        li = sum(1 for _, la, _ in launches if la <= a)
        print(f"  {f:32s} {(b - a) / 1e3:10.1f} us at {(a - t0) / 1e6:10.3f} ms (after launch #{li})")
    if kpath:
        ks = _rows(kpath)
        hw = sorted(int(r["Start_Timestamp"]) for r in ks if "host_wait" in r.get("Kernel_Name", ""))
        if hw:
            gaps = [(b - a) / 1e6 for a, b in zip(hw, hw[1:])]
            print("host_wait kernel starts (replay heads), ms between consecutive ones:")
            print("  " + " ".join(f"{g:.3f}" for g in gaps))


if __name__ == "__main__":
    if len(sys.argv) < 3 or sys.argv[1] not in ("queues", "api"):
        print(__doc__)
        sys.exit(2)
    if sys.argv[1] == "queues":
        queues(sys.argv[2])
    else:
        api(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
