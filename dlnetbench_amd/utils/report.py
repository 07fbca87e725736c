"""Parse benchmark output into documents and pandas DataFrames.

Reference: plots/parser.py walks SbatchMan jobs and parses the external
ccutils stdout format (MPIOutputParser) into DP / FSDP DataFrames
(extract_dp_metrics_df :139-196, extract_fsdp_metrics_df :19-100,
validate_dp_output :102-136). ccutils is not available, so the native runtime
prints a self-describing block

    <<<DLNB_REPORT_BEGIN <section>>>>
    {"section": ..., "title": ..., "global": {...}, "ranks": [{...}, ...]}
    <<<DLNB_REPORT_END <section>>>>

and this module turns it into the same columns (plus dlnb extras). The
collective-library knobs the reference recorded as SbatchMan job variables
(protocol / algorithm / channels / threads, parser.py:151-154) are taken
from the run's recorded environment (NCCL_PROTO, NCCL_ALGO,
NCCL_MIN_NCHANNELS, NCCL_NTHREADS) unless job_vars overrides them.
"""
from __future__ import annotations

import argparse
import glob
import json
import re
import sys
from typing import Dict, Iterable, List, Optional, Tuple

_BLOCK = re.compile(r"<<<DLNB_REPORT_BEGIN (\S+)>>>\n(.*?)\n<<<DLNB_REPORT_END \1>>>", re.S)


def parse_output(text: str) -> Dict[str, dict]:
    """All report sections found in a stdout capture, keyed by section id."""
    return {m.group(1): json.loads(m.group(2)) for m in _BLOCK.finditer(text)}


def load_reports(paths: Iterable[str]) -> List[dict]:
    docs = []
    for p in paths:
        with open(p) as f:
            text = f.read()
        try:
            docs.append(json.loads(text))  # a --json file
            continue
        except json.JSONDecodeError:
            pass
        docs.extend(parse_output(text).values())
    return docs


def validate(doc: dict, expected_world: Optional[int] = None, nodes: Optional[int] = None) -> List[str]:
    """Rank/host sanity checks (reference validate_dp_output): returns warnings."""
    warn = []
    ranks = sorted(r.get("rank", i) for i, r in enumerate(doc.get("ranks", [])))
    world = expected_world if expected_world is not None else doc["global"].get("world_size")
    if world is not None and ranks != list(range(world)):
        warn.append(f"[VALIDATION][RANK] expected ranks 0..{world - 1}, got {ranks}")
    if nodes is not None:
        hosts = {r.get("hostname") for r in doc.get("ranks", [])}
        if len(hosts) != nodes:
            warn.append(f"[VALIDATION][HOSTNAME] expected {nodes} hosts, got {len(hosts)}: {sorted(hosts)}")
    return warn


def _knobs(doc: dict, job_vars: Optional[dict]) -> dict:
    env = doc["global"].get("dlnb", {}).get("env", {})
    jv = job_vars or {}
    return {
        "protocol": jv.get("protocol", env.get("NCCL_PROTO")),
        "algorithm": jv.get("algorithm", env.get("NCCL_ALGO")),
        "channels": jv.get("channels", env.get("NCCL_MIN_NCHANNELS")),
        "threads": jv.get("threads", env.get("NCCL_NTHREADS")),
    }


def dp_dataframe(doc: dict, job_vars: Optional[dict] = None, network: str = "mi355x"):
    import pandas as pd
    g = doc["global"]
    base = {
        "network": network, "world_size": g["world_size"], "model_name": g["model_name"],
        "local_batch_size": g["local_batch_size"], "num_buckets": g["num_buckets"], **_knobs(doc, job_vars),
        "fwd_rt_whole_model": g["fwd_rt_whole_model"], "bwd_rt_per_bucket": g["bwd_rt_per_bucket"],
        "msg_size_avg_bytes": g["msg_size_avg_bytes"], "msg_size_std_bytes": g["msg_size_std_bytes"],
        "backend": g["backend"], "schedule": g.get("dlnb", {}).get("schedule"),
    }
    rows = []
    for r in doc["ranks"]:
        energy = r.get("energy_consumed") or [None] * len(r["runtimes"])
        for i, (rt, bt) in enumerate(zip(r["runtimes"], r["barrier_time"])):
            rows.append({**base, "rank": r["rank"], "hostname": r.get("hostname"), "run": i, "runtime": rt,
                         "barrier_time": bt, "energy_consumed": energy[i] if i < len(energy) else None})
    return pd.DataFrame(rows)


def fsdp_dataframes(doc: dict, job_vars: Optional[dict] = None, network: str = "mi355x") -> Tuple:
    """(runtime_df, comm_df) with the reference's columns (parser.py:19-100).

    comm_df has one row per rank x run x unit: allgather_wait_fwd for units
    1..U-1 (the wait before that unit's forward), allgather_wait_bwd for
    units U-2..0, reduce_scatter for every unit (backward order U-1..0)."""
    import pandas as pd
    g = doc["global"]
    U = g["num_units"]
    base = {
        "network": network, "world_size": g["world_size"], "sharding_factor": g["sharding_factor"],
        "num_replicas": g["num_replicas"], "model_name": g["model_name"], "model_size_bytes": g["model_size_bytes"],
        "local_batch_size": g["local_batch_size"], "num_units": U,
        "fwd_time_per_unit_us": g["fwd_time_per_unit_us"], "bwd_time_per_unit_us": g["bwd_time_per_unit_us"],
        "allgather_msg_size_bytes": g["allgather_msg_size_bytes"],
        "reducescatter_msg_size_bytes": g["reducescatter_msg_size_bytes"], **_knobs(doc, job_vars),
    }
    rt_rows, comm_rows = [], []
    for r in doc["ranks"]:
        runs = len(r["runtime"])
        for i in range(runs):
            rt_rows.append({**base, "rank": r["rank"], "hostname": r.get("hostname"), "run": i,
                            "runtime": r["runtime"][i],
                            "allgather": r["allgather"][i] if i < len(r["allgather"]) else None,
                            "barrier": r["barrier"][i] if i < len(r["barrier"]) else 0})
            wf = r["allgather_wait_fwd"][i * (U - 1):(i + 1) * (U - 1)]
            wb = r["allgather_wait_bwd"][i * (U - 1):(i + 1) * (U - 1)]
            rs = r["reduce_scatter"][i * U:(i + 1) * U]
            for u in range(U):
                comm_rows.append({**base, "rank": r["rank"], "hostname": r.get("hostname"), "run": i, "unit_idx": u,
                                  "allgather_wait_fwd": wf[u - 1] if 1 <= u <= len(wf) else 0.0,
                                  "allgather_wait_bwd": wb[U - 2 - u] if u <= U - 2 and U - 2 - u < len(wb) else 0.0,
                                  "reduce_scatter": rs[U - 1 - u] if U - 1 - u < len(rs) else 0.0})
    return pd.DataFrame(rt_rows), pd.DataFrame(comm_rows)


def hybrid_dataframe(doc: dict, network: str = "mi355x"):
    """One row per rank x run for dp_pp / dp_pp_tp / dp_pp_ep / dp_pp_tp_ep sections."""
    import pandas as pd
    g = doc["global"]
    rows = []
    keys = [k for k in ("pp_comm_time", "dp_comm_time", "tp_comm_time", "ep_comm_time", "dp_ep_comm_time",
                        "pp_mirror_time")]
    for r in doc["ranks"]:
        runs = len(r["runtimes"])
        for i in range(runs):
            row = {"network": network, "section": doc["section"], "model_name": g["model_name"],
                   "world_size": g["world_size"], "num_stages": g["num_stages"],
                   "num_microbatches": g["num_microbatches"], "dp_size": g["dp_size"], "rank": r["rank"],
                   "stage_id": r.get("stage_id"), "run": i, "runtime": r["runtimes"][i],
                   "pp_schedule": g.get("pp_schedule", "gpipe"), "ep_imbalance": g.get("ep_imbalance", 0.0),
                   "ep_id": r.get("ep_id")}
            for k in keys:
                if k in r and r[k]:
                    per = len(r[k]) // runs
                    row[k] = sum(r[k][i * per:(i + 1) * per])
            rows.append(row)
    return pd.DataFrame(rows)


def cp_dataframe(doc: dict, network: str = "mi355x"):
    """One row per rank x run for dp_cp sections (hybrid_cp: per-iteration CP / DP communication sums)."""
    import pandas as pd
    g = doc["global"]
    rows = []
    for r in doc["ranks"]:
        for i, rt in enumerate(r["runtimes"]):
            row = {"network": network, "section": doc["section"], "model_name": g["model_name"],
                   "world_size": g["world_size"], "num_cp_shards": g["num_cp_shards"], "cp_algo": g["cp_algo"],
                   "dp_size": g["dp_size"], "rank": r["rank"], "cp_id": r.get("cp_id"), "run": i, "runtime": rt}
            for k in ("cp_comm_time", "cp_exposed_time", "dp_comm_time", "dp_exposed_time"):
                v = r.get(k) or []
                row[k] = v[i] if i < len(v) else 0.0
            rows.append(row)
    return pd.DataFrame(rows)


def summary(doc: dict) -> dict:
    """Headline numbers of one run: iteration stats + per-collective bus bandwidth."""
    g = doc["global"]
    it = g.get("dlnb", {}).get("iteration", {})
    out = {"section": doc["section"], "model": g.get("model_name"), "world_size": g.get("world_size"),
           "backend": g.get("backend"), "median_ms": it.get("median_ms"), "floor_ms": it.get("compute_floor_ms")}
    bw: Dict[str, List[float]] = {}
    for r in doc["ranks"]:
        for k, v in r.get("comm", {}).items():
            if "busbw_GBps" in v:
                bw.setdefault(k, []).append(v["busbw_GBps"])
    out["busbw_GBps"] = {k: sum(v) / len(v) for k, v in bw.items()}
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Turn dlnb outputs into CSV")
    ap.add_argument("inputs", nargs="+", help="stdout captures or --json files (globs allowed)")
    ap.add_argument("--csv", default=None)
    a = ap.parse_args(argv)
    paths = [p for pat in a.inputs for p in (glob.glob(pat) or [pat])]
    docs = load_reports(paths)
    import pandas as pd
    frames = []
    for d in docs:
        for w in validate(d):
            print(w, file=sys.stderr)
        if d["section"] == "dp":
            frames.append(dp_dataframe(d))
        elif d["section"] == "fsdp":
            frames.append(fsdp_dataframes(d)[0])
        elif d["section"] == "dp_cp":
            frames.append(cp_dataframe(d))
        else:
            frames.append(hybrid_dataframe(d))
        print(json.dumps(summary(d)))
    if a.csv and frames:
        pd.concat(frames, ignore_index=True).to_csv(a.csv, index=False)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
