"""Table of scripts/probes/deadline_stream.sh: TF/s, clock, MFMA busy of the
deadline GEMM dispatches (launches 2-5; the first one ramps the clock)."""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
print("| dtype | shape | kernel | TF/s (launches 2-5) | clock GHz | MFMA busy |")
print("|---|---|---|---:|---:|---:|")
for d in sorted(glob.glob(os.path.join(root, "*_s[0-9]"))):
    tag = os.path.basename(d)
    dt, shape, s = tag.split("_")
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not cc or not kt:
        continue
    dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(kt[0]))}
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(cc[0])):
        if "gemm" in r["Kernel_Name"]:
            agg[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    rows = []
    for k in sorted(agg)[1:]:
        c, t = agg[k], dur.get(str(k), 0) * 1e-9
        if not t:
            continue
        fl = (c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) + c.get("SQ_INSTS_VALU_MFMA_MOPS_F8", 0)) * 512
        gui = c.get("GRBM_GUI_ACTIVE", 0) / 8 / t
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui * t * 256 * 4) if gui else 0
        rows.append((fl / t / 1e12, gui / 1e9, busy))
    if rows:
        tf = sorted(r[0] for r in rows)
        print(f"| {dt} | {shape} | { {'s0': 'per-tile', 's1': 'stream', 's2': 'per-tile uniform'}.get(s, 'probe ' + s)} | {tf[0]:.0f}-{tf[-1]:.0f} | "
              f"{sum(r[1] for r in rows) / len(rows):.2f} | {sum(r[2] for r in rows) / len(rows):.3f} |")
