"""Summarise rocprofv3 CSV output (kernel stats / kernel trace / PMC) as markdown.

    python -m dlnetbench_amd.tools.prof_summary gpurun_out/prof_fsdp [--pmc gpurun_out/pmc_gemm] > profiles/x.md
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re


def _short(name: str) -> str:
    name = re.sub(r"\(anonymous namespace\)::", "", name)
    name = re.sub(r"\(.*", "", name)
    return name[:90]


def kernel_stats(d: str) -> str:
    files = glob.glob(os.path.join(d, "*kernel_stats.csv"))
    if not files:
        return ""
    rows = list(csv.DictReader(open(files[0])))
    out = ["| kernel | calls | total ms | avg us | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:15]:
        out.append(f"| `{_short(r['Name'])}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    return "\n".join(out)


def pmc(d: str) -> str:
    files = glob.glob(os.path.join(d, "*counter_collection.csv"))
    if not files:
        return ""
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = collections.defaultdict(float)
    seen = set()
    for r in csv.DictReader(open(files[0])):
        k = _short(r["Kernel_Name"])
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        key = (k, r["Dispatch_Id"])
        if key not in seen:
            seen.add(key)
            dur[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
    names = sorted({c for v in agg.values() for c in v})
    out = ["| kernel | " + " | ".join(names) + " | ms |", "|---|" + "---:|" * (len(names) + 1)]
    for k, v in agg.items():
        out.append(f"| `{k}` | " + " | ".join(f"{v.get(n, 0):.3g}" for n in names) + f" | {dur[k]:.2f} |")
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace_dir", nargs="?")
    ap.add_argument("--pmc", default=None)
    ap.add_argument("--title", default="rocprofv3 summary")
    a = ap.parse_args(argv)
    print(f"# {a.title}\n")
    if a.trace_dir:
        print("## Kernel time (rocprofv3 --kernel-trace --stats)\n")
        print(kernel_stats(a.trace_dir) + "\n")
    if a.pmc:
        print("## Counters (rocprofv3 --pmc), summed over dispatches\n")
        print(pmc(a.pmc) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
