"""TFLOP/s per dispatch from a rocprofv3 --pmc run with SQ_INSTS_VALU_MFMA_MOPS_BF16
(x 512 FLOP) and the kernel trace: python scripts/probes/pmc_rate.py <dir> [name-filter]."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else "gemm"
rows = list(csv.DictReader(open(glob.glob(f"{d}/*counter_collection.csv")[0])))
kt = list(csv.DictReader(open(glob.glob(f"{d}/*kernel_trace.csv")[0])))
dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in kt}
agg = collections.defaultdict(lambda: collections.defaultdict(float))
names = {}
for r in rows:
    if filt in r["Kernel_Name"]:
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"][:60]
for k, c in agg.items():
    t = dur.get(k, 0) * 1e-9
    fl = c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0) * 512
    clk = c.get("GRBM_GUI_ACTIVE", 0) / 8 / t / 1e9 if t else 0
    print(f"{k:>4} {names[k]} {t * 1e3:8.2f} ms {fl / t / 1e12 if t else 0:8.1f} TF/s  clk~{clk:.2f} GHz")
