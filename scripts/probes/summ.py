#!/usr/bin/env python3
"""Summaries of the round-5 lane probes: python scripts/probes/summ.py <dir> <name>..."""
import json
import statistics as st
import sys

d = sys.argv[1]
for f in sys.argv[2:]:
    try:
        j = json.load(open(f"{d}/{f}.json"))
    except Exception as e:  # noqa: BLE001
        print(f, "missing", e)
        continue
    if "metric" in j:  # a bench.py line
        print(f, j["value"], "exposed", j["exposed_comm_ms"], "absorbed", j.get("chain_absorbed_ms_per_iter"),
              "runs", j["per_run_ms"])
        continue
    g = j["global"]["dlnb"]
    it = g["iteration"]
    r = j["ranks"][0]
    cc = g.get("chain_capped") or {}
    b = r.get("barrier_time") or r.get("barrier")
    sp = r.get("device_span_time")
    lg = g.get("lane_graphs") or {}
    print(f, "med %.4f floor %.4f" % (it["median_ms"], it["compute_floor_ms"]), "barrier %.4f" % (st.mean(b) * 1e3),
          "span-floor %s" % ("%.4f" % (st.mean(sp) * 1e3 - it["compute_floor_ms"]) if sp else None),
          "capped %.2f/%.4f absorbed %.4f" % (cc.get("tasks_per_iter_max", 0), cc.get("ms_per_iter_max", 0),
                                              cc.get("absorbed_ms_per_iter_max", 0)),
          "lanes", lg.get("enabled"), lg.get("program_join"), "unc", g["compute"].get("wallclock_uncertainty_ppm"))
