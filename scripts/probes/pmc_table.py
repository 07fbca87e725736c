"""Per-kernel PMC table from rocprofv3 --pmc runs (one directory per pass):
mean duration, clock, TFLOP/s (MFMA MOPS x 512) and each counter as a rate
(per ns of kernel time, per CU where the counter is per-SE/CU summed).
usage: python scripts/probes/pmc_table.py <dir> [<dir> ...]"""
import collections
import csv
import glob
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    rows = list(csv.DictReader(open(glob.glob(f"{d}/*counter_collection.csv")[0])))
    kt = list(csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0])))
    dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt}
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in rows:
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        name[r["Dispatch_Id"]] = r["Kernel_Name"][:48]
    for k, c in per.items():
        nm = name[k]
        acc[nm]["dur_ns"].append(dur.get(k, 0))
        for cn, v in c.items():
            acc[nm][cn].append(v)
for nm, c in acc.items():
    if len(c["dur_ns"]) < 4:
        continue
    mean = {k: sum(v) / len(v) for k, v in c.items()}
    t = sum(c["dur_ns"]) / len(c["dur_ns"])
    gui = mean.get("GRBM_GUI_ACTIVE", 0) / 8
    out = {"kernel": nm, "n": len(c["dur_ns"]), "ms": round(t / 1e6, 3), "clk_GHz": round(gui / t, 3) if t else 0}
    for mops in ("SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_INSTS_VALU_MFMA_MOPS_F8"):
        if mops in mean:
            out["TFLOPs"] = round(mean[mops] * 512 / t / 1e3, 1)
    for k, v in sorted(mean.items()):
        if k not in ("dur_ns", "GRBM_GUI_ACTIVE"):
            out[k] = round(v / gui, 3) if gui else v  # per GPU-clock cycle
    print(out)
