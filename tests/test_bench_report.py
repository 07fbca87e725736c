"""tools/bench_report.py: scaling table from bench.py result lines."""
from __future__ import annotations

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dlnetbench_amd.tools import bench_report  # noqa: E402


def _line(n, ms, ag=None, c5=None, xgmi=None, hx=None):
    d = {"metric": "m", "value": ms, "unit": "ms", "n_gpus": n, "ms_per_step": ms, "exposed_comm_ms": ms - 2814.75,
         "effective_busbw_GBps": {"allgather": ag, "reduce_scatter": ag}}
    if c5 is not None:
        d["comm_bound"] = {"ms_per_step": c5, "allreduce_busbw_GBps": None if n == 1 else 300.0,
                           "rccl_default_ctas": {"ms_per_step": c5 - 0.5}}
    if xgmi is not None:
        d["comm_bound_xgmi"] = {"ms_per_step": xgmi, "speedup_vs_comm_bound": round(c5 / xgmi, 4)}
    if hx is not None:
        d["headline_xgmi"] = {"busbw_ratio_vs_headline": {"allgather": hx, "reduce_scatter": hx}}
    return json.dumps(d)


def test_scaling_rows_sorted_with_efficiency(tmp_path):
    # stdout of three runs in arbitrary order, with non-JSON noise (banners) in between
    p = tmp_path / "runs.txt"
    p.write_text("\n".join([
        "RCCL version 2.x", _line(8, 2830.0, ag=250.0, c5=9.0, xgmi=7.5, hx=1.3),
        _line(1, 2816.5, c5=7.25), "{not json", _line(2, 2820.0, ag=110.0, c5=14.5, xgmi=14.2, hx=1.05)]))
    rs = bench_report.rows(bench_report.load([str(p)]))
    assert [r["n_gpus"] for r in rs] == [1, 2, 8]
    assert rs[0]["efficiency"] == 1.0
    assert rs[2]["efficiency"] == round(2816.5 / 2830.0, 4)
    assert rs[0]["ag_busbw_GBps"] is None and rs[2]["ag_busbw_GBps"] == 250.0
    assert rs[2]["c5_uncapped_ms"] == 8.5 and rs[2]["c5_xgmi_speedup"] == round(9.0 / 7.5, 4)
    assert rs[2]["fsdp_xgmi_ag_ratio"] == 1.3 and rs[0]["c5_xgmi_ms"] is None
    md = bench_report.markdown(rs)
    assert md.count("\n") == 5 and "| 8 |" in md and "—" in md


def test_cli_json_array_and_csv(tmp_path, capsys):
    p = tmp_path / "a.json"
    p.write_text("[" + ",".join([_line(4, 2818.0, ag=180.0), _line(1, 2816.0)]) + "]")
    out = tmp_path / "s.csv"
    assert bench_report.main([str(p), "--csv", str(out)]) == 0
    text = capsys.readouterr().out
    assert text.splitlines()[0].startswith("| n_gpus | ms_per_step | efficiency")
    rows = out.read_text().splitlines()
    assert rows[0].startswith("n_gpus,ms_per_step,efficiency") and len(rows) == 3


def test_failed_and_fallback_lines(tmp_path):
    """A line whose headline failed (value null) gets no efficiency and does not become the N = 1 reference;
    a line timed on the fallback backend says so."""
    fail = {"metric": "m", "value": None, "unit": "ms", "n_gpus": 2, "ms_per_step": None, "error": "headline failed"}
    fb = json.loads(_line(8, 2820.0))
    fb["config"] = {"backend": "XGMI"}
    fb["headline_fallback"] = {"backend": "xgmi", "primary_backend": "auto", "primary_error": "rccl init"}
    p = tmp_path / "r.txt"
    p.write_text("\n".join([json.dumps(fail), _line(1, 2816.0), json.dumps(fb)]))
    rs = bench_report.rows(bench_report.load([str(p)]))
    assert [r["n_gpus"] for r in rs] == [1, 2, 8]
    assert rs[1]["efficiency"] is None and rs[2]["efficiency"] == round(2816.0 / 2820.0, 4)
    assert rs[2]["backend"] == "XGMI" and rs[2]["fallback"] and not rs[0]["fallback"]


def test_no_lines_is_an_error(tmp_path):
    p = tmp_path / "empty.txt"
    p.write_text("nothing here\n")
    assert bench_report.main([str(p)]) == 1


def test_exactness_and_hybrid_columns():
    d = json.loads(_line(8, 2816.0, ag=300.0, c5=7.4))
    d["comm_bound"]["geometric_buckets"] = {"ms_per_step": 7.25}
    d["exact"] = {"rccl": True, "xgmi": False, "rccl_eager": True}
    d["exact_detail"] = {"xgmi_release": None}
    d["rccl_nranks"] = {"fsdp/unit/0": 8}
    d["hybrid_3d"] = {"ms_per_step": 3900.0, "vs_floor": 1.02}
    d["hybrid_3d_moe"] = {"ms_per_step": 15000.0, "vs_floor": 1.1, "ep_overlap": {"ms_per_step": 13600.0}}
    d["predicted_ms"] = 2815.9
    d["phase_seconds"] = {"headline": 72.5, "total": 231.4}
    d["link_bench"] = {"rccl": {"all_reduce": {"8388608": {"busbw_GBps": 250.0}, "67108864": {"busbw_GBps": 310.0}}},
                       "xgmi_registered": {"error": "x"}}
    r = bench_report.rows([d])[0]
    assert r["c4_overlap_ms"] == 13600.0 and r["predicted_ms"] == 2815.9
    assert r["link_ar_busbw_rccl"] == 310.0 and r["link_ar_busbw_xgmi"] is None
    assert r["c5_geometric_ms"] == 7.25 and r["exact_rccl"] is True and r["exact_xgmi"] is False
    assert r["rccl_nranks"] == 8 and r["c3_vs_floor"] == 1.02 and r["c4_ms"] == 15000.0
    assert r["wall_s"] == 231.4
    r1 = bench_report.rows([json.loads(_line(1, 2816.0))])[0]
    assert r1["exact_rccl"] is None and r1["rccl_nranks"] is None and r1["c3_ms"] is None


def test_nested_scaling_record(tmp_path):
    """A driver-style record that nests the per-N lines (as dicts or inside a captured stdout string)."""
    one = json.loads(_line(1, 2816.0))
    eight = json.loads(_line(8, 2818.0))
    doc = {"runs": [{"n": 1, "result": one}, {"n": 8, "stdout": "[bench] noise\n" + json.dumps(eight) + "\n"}]}
    p = tmp_path / "scale.json"
    p.write_text(json.dumps(doc, indent=1))
    assert [d["n_gpus"] for d in bench_report.load([str(p)])] == [1, 8]

