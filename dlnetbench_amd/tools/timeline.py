"""Summaries of a device timeline (``--timeline PATH``, csrc/src/timeline.cpp).

    python -m dlnetbench_amd timeline trace.json [--json] [--check]

Per rank and iteration: the span from the first to the last traced op,
compute busy time, communication busy time, how much of the communication ran
while compute was busy on the same rank (hidden) and how much did not
(exposed), plus per-operation totals. ``--check`` verifies the trace is
well-formed: spans of one stream do not overlap (a stream is in order) and
every rank has events of every kept iteration.

The reference reports only per-phase host timer vectors; this
is the view the reference's ``barrier_time`` ("exposed communication") is a
one-number summary of.
"""
from __future__ import annotations

import argparse
import json
from collections import defaultdict
from typing import Dict, List, Tuple

Interval = Tuple[float, float]


def _union(iv: List[Interval]) -> List[Interval]:
    out: List[Interval] = []
    for a, b in sorted(iv):
        if out and a <= out[-1][1]:
            out[-1] = (out[-1][0], max(out[-1][1], b))
        else:
            out.append((a, b))
    return out


def _length(iv: List[Interval]) -> float:
    return sum(b - a for a, b in iv)


def _intersect(x: List[Interval], y: List[Interval]) -> float:
    """Total length of the intersection of two unions of intervals."""
    i = j = 0
    tot = 0.0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if b > a:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def load(path: str) -> List[dict]:
    with open(path) as f:
        doc = json.load(f)
    return [e for e in doc["traceEvents"] if e.get("ph") == "X"]


def summarize(events: List[dict]) -> Dict[str, dict]:
    """{rank: {iter: {...}}} in milliseconds."""
    by = defaultdict(list)
    for e in events:
        by[(e["pid"], e["args"]["iter"])].append(e)
    out: Dict[str, dict] = defaultdict(dict)
    for (pid, it), evs in sorted(by.items()):
        host = [e for e in evs if e["cat"] == "host"]
        edges = {e["name"]: e["ts"] for e in evs if e["cat"] == "edge"}
        evs = [e for e in evs if e["cat"] not in ("host", "edge")]
        if not evs:
            continue
        comp = _union([(e["ts"], e["ts"] + e["dur"]) for e in evs if e["cat"] == "compute"])
        comm = _union([(e["ts"], e["ts"] + e["dur"]) for e in evs if e["cat"] in ("comm", "p2p")])
        t0 = min(e["ts"] for e in evs)
        t1 = max(e["ts"] + e["dur"] for e in evs)
        hidden = _intersect(comp, comm)
        ops: Dict[str, dict] = defaultdict(lambda: {"count": 0, "ms": 0.0, "bytes": 0.0})
        for e in evs:
            if e["cat"] == "compute":
                continue
            key = e["name"].split(" ")[0]
            ops[key]["count"] += 1
            ops[key]["ms"] += e["dur"] / 1e3
            ops[key]["bytes"] += float(e["args"].get("bytes", 0.0))
        out[str(pid)][str(it)] = {
            "span_ms": (t1 - t0) / 1e3,
            "compute_busy_ms": _length(comp) / 1e3,
            "comm_busy_ms": _length(comm) / 1e3,
            "comm_hidden_ms": hidden / 1e3,
            "comm_exposed_ms": (_length(comm) - hidden) / 1e3,
            "compute_idle_ms": (t1 - t0 - _length(comp)) / 1e3,
            "ops": {k: dict(v) for k, v in sorted(ops.items())},
        }
        if host:
            # the iteration as the host timed it, and what it adds to the device span
            # (graph launch / enqueue before the first op, completion detection after the last)
            h = host[0]
            r = out[str(pid)][str(it)]
            r["host_ms"] = h["dur"] / 1e3
            r["launch_ms"] = (t0 - h["ts"]) / 1e3
            r["completion_ms"] = (h["ts"] + h["dur"] - t1) / 1e3
            if len(edges) == 2:
                # DLNB_TIMELINE_EDGES=1: stamps on the launch stream around the graph launch
                e0, e1 = edges["before graph launch"], edges["after graph launch"]
                r["edges"] = {"submit_ms": (e0 - h["ts"]) / 1e3, "graph_start_ms": (t0 - e0) / 1e3,
                              "graph_join_ms": (e1 - t1) / 1e3, "detect_ms": (h["ts"] + h["dur"] - e1) / 1e3}
    return dict(out)


def check(events: List[dict]) -> List[str]:
    """Problems found (empty = well-formed)."""
    bad: List[str] = []
    lanes = defaultdict(list)
    iters = defaultdict(set)
    for e in events:
        if e["dur"] < 0:
            bad.append(f"negative duration: {e}")
        lanes[(e["pid"], e["tid"], e["args"]["iter"])].append((e["ts"], e["ts"] + e["dur"], e["name"]))
        iters[e["pid"]].add(e["args"]["iter"])
    for key, iv in lanes.items():
        iv.sort()
        for (a0, a1, an), (b0, b1, bn) in zip(iv, iv[1:]):
            if b0 < a1 - 2e-3:  # the trace rounds to 1 ns (either end)
                bad.append(f"rank {key[0]} stream {key[1]} iter {key[2]}: '{bn}' starts before '{an}' ends")
    want = set().union(*iters.values()) if iters else set()
    for pid, its in iters.items():
        if its != want:
            bad.append(f"rank {pid} has iterations {sorted(its)}, others {sorted(want)}")
    return bad


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("trace")
    ap.add_argument("--json", action="store_true", help="print the summary as JSON")
    ap.add_argument("--check", action="store_true", help="verify in-order streams and complete iterations")
    a = ap.parse_args(argv)
    ev = load(a.trace)
    if a.check:
        bad = check(ev)
        for b in bad[:20]:
            print("timeline check:", b)
        if bad:
            return 1
    s = summarize(ev)
    if a.json:
        print(json.dumps(s, indent=1))
        return 0
    print(f"{'rank':>4} {'iter':>4} {'span ms':>10} {'compute':>10} {'comm':>10} {'hidden':>10} {'exposed':>10}"
          f" {'host ms':>10} {'launch':>8} {'complete':>8}")
    for pid, its in s.items():
        for it, r in its.items():
            host = (f" {r['host_ms']:10.3f} {r['launch_ms']:8.3f} {r['completion_ms']:8.3f}" if "host_ms" in r
                    else "")
            if "edges" in r:
                host += " " + " ".join(f"{k[:-3]}={v:.3f}" for k, v in r["edges"].items())
            print(f"{pid:>4} {it:>4} {r['span_ms']:10.3f} {r['compute_busy_ms']:10.3f} {r['comm_busy_ms']:10.3f} "
                  f"{r['comm_hidden_ms']:10.3f} {r['comm_exposed_ms']:10.3f}{host}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
