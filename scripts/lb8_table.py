"""Markdown table from scripts/loopback_w8.sh outputs (gpurun_out/lb8_*.json)."""
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
print("| run | W | median ms | compute floor ms (scaled) | collectives of rank 0: kind (group) bytes/op x ops |")
print("|---|---:|---:|---:|---|")
for p in sorted(glob.glob(os.path.join(d, "lb8_*.json"))):
    doc = json.load(open(p))
    g = doc["global"]
    it = g["dlnb"]["iteration"]
    comm = doc["ranks"][0].get("comm", {})
    kinds = "; ".join(f"{k} ({v['nranks']}) {v['bytes_per_op'] / 1e6:.1f} MB x {v['ops']}" for k, v in comm.items())
    name = os.path.basename(p)[4:-5]
    print(f"| {name} | {g['world_size']} | {it['median_ms']:.1f} | {it['compute_floor_ms']:.1f} | {kinds} |")
