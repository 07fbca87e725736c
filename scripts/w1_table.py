"""Markdown table from scripts/strategies_w1.sh outputs (gpurun_out/w1_*.json)."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
print("| run | median ms | compute floor ms | over floor |")
print("|---|---:|---:|---:|")
for p in sorted(glob.glob(os.path.join(d, "w1_*.json"))):
    doc = json.load(open(p))
    it = doc["global"]["dlnb"]["iteration"]
    m, f = it["median_ms"], it["compute_floor_ms"]
    name = os.path.basename(p)[3:-5]
    print(f"| {name} | {m:.3f} | {f:.3f} | {m - f:.3f} ms ({(m / f - 1) * 100:.2f} %) |")
