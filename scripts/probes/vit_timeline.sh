#!/bin/bash
# Kernel-trace timeline of the comm-bound ViT-H DP iteration (bench.py's comm_bound block).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/vt
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/vt -o run -- \
  build/bin/dp vit_h_32_float8 8 . --no-topology --quiet -w 5 -r 30 --graph --json gpurun_out/vt/report.json \
  > gpurun_out/vt/log.txt 2>&1 || exit $?
f=$(find gpurun_out/vt -name '*kernel_trace.csv' | head -1)
python3 scripts/probes/vit_timeline.py "$f" 2376.55 594.1375 > gpurun_out/vt/timeline.txt
python3 -c "import json; d=json.load(open('gpurun_out/vt/report.json'))['global']['dlnb']['iteration']; print(d['timed_ms_per_iter'], d['median_ms'], d['compute_floor_ms'])" >> gpurun_out/vt/timeline.txt
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))[-3000:]
with open("gpurun_out/vt/trace_tail.csv", "w", newline="") as f:
    w = csv.writer(f)
    w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Queue_Id"])
    for r in rows:
        w.writerow([r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-80:], r["Start_Timestamp"], r["End_Timestamp"], r.get("Queue_Id", "?")])
PY
rm -f "$f"
