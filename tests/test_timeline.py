"""--timeline: the device timeline of every rank (csrc/src/timeline.cpp) and its
summary tool (dlnetbench_amd/tools/timeline.py)."""
from __future__ import annotations

import json
import os
import subprocess
import sys
from collections import Counter

import pytest

from dlnetbench_amd.tools import timeline as tlt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "tests", "data")
BIN = os.path.join(ROOT, "build", "bin")


def _launch(n, args, timeout=120):
    cmd = [sys.executable, "-m", "dlnetbench_amd.utils.launch", "-n", str(n), "--timeout", str(timeout)] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 30, cwd=ROOT,
                          env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def _events(path):
    with open(path) as f:
        doc = json.load(f)
    return doc, [e for e in doc["traceEvents"] if e["ph"] == "X"]


def test_fsdp_timeline_two_processes(tmp_path):
    """2 ranks on the shm backend, 4 units, 3 timed runs, the last 2 kept:
    per rank and iteration 2U-1 all-gathers, U reduce-scatters and 2U compute
    tasks, every stream in order, one process per rank in the trace."""
    out, rep = tmp_path / "tl.json", tmp_path / "r.json"
    p = _launch(2, [os.path.join(BIN, "fsdp"), "tiny_dense_8_bfloat16", "4", "2", DATA, "--backend", "cpu",
                    "--compute", "sleep", "-w", "1", "-r", "3", "--quiet", "--timeline", str(out), "--json", str(rep)])
    assert p.returncode == 0, p.stderr[-2000:]
    doc, ev = _events(out)
    assert tlt.check(ev) == []
    c = Counter((e["pid"], e["args"]["iter"], e["name"].split(" ")[0]) for e in ev)
    for pid in (0, 1):
        for it in (1, 2):
            assert c[(pid, it, "all_gather")] == 7 and c[(pid, it, "reduce_scatter")] == 4
            assert c[(pid, it, "compute")] == 8
    assert {e["args"]["iter"] for e in ev} == {1, 2}
    names = {m["args"]["name"] for m in doc["traceEvents"] if m["ph"] == "M" and m["name"] == "thread_name"}
    assert "compute" in names and any(n.startswith("comm: fsdp/") for n in names)
    from dlnetbench_amd.tools import plots
    drawn = plots.plot_timeline(str(out), str(tmp_path / "tl.png"))
    assert drawn == {"comm": 2 * 11, "compute": 2 * 8, "host": 2} and (tmp_path / "tl.png").stat().st_size > 0
    g = json.loads(rep.read_text())["global"]["dlnb"]["timeline"]
    assert g["events"] == len(ev) and g["truncated"] is False and g["path"] == str(out)
    s = tlt.summarize(ev)
    for pid in ("0", "1"):
        r = s[pid]["2"]
        assert r["comm_busy_ms"] > 0 and r["compute_busy_ms"] > 0
        assert r["comm_hidden_ms"] + r["comm_exposed_ms"] == pytest.approx(r["comm_busy_ms"])
        # the host's view of the iteration (what the runner times) brackets the device spans
        assert r["host_ms"] >= r["span_ms"] - 0.05 and r["launch_ms"] > -0.05 and r["completion_ms"] > -0.05
        assert r["ops"]["all_gather"]["count"] == 7 and r["ops"]["all_gather"]["bytes"] > 0


def test_pipeline_timeline_p2p_groups(tmp_path):
    """hybrid_3d_moe 1F1B as 4 loopback-cpu rank threads: each grouped
    send/recv is one p2p span, the expert all-to-alls sit on the compute
    stream (eager), every rank thread lands in the one trace rank 0 writes."""
    out = tmp_path / "tl.json"
    p = subprocess.run([os.path.join(BIN, "hybrid_3d_moe"), "tiny_moe_8_bfloat16", "2", "4", "2", DATA,
                        "--backend", "loopback-cpu", "--ranks", "4", "--compute", "sleep", "-w", "1", "-r", "2",
                        "--quiet", "--pp-schedule", "1f1b", "--timeline", str(out), "--timeline-iters", "0"],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    doc, ev = _events(out)
    assert tlt.check(ev) == []
    assert {e["pid"] for e in ev} == {0, 1, 2, 3}
    p2p = [e for e in ev if e["cat"] == "p2p"]
    assert p2p and all(e["args"]["bytes"] > 0 for e in p2p)
    assert any("," in e["args"]["ops"] for e in p2p)  # a send and a recv in one group
    lanes = {(m["pid"], m["tid"]): m["args"]["name"] for m in doc["traceEvents"]
             if m["ph"] == "M" and m["name"] == "thread_name"}
    # (eager: the expert all-to-alls stay on the compute stream; lane graphs put them on the inner lane)
    assert all(lanes[(e["pid"], e["tid"])] == "compute" for e in ev if e["name"].startswith("all_to_all"))
    assert {e["args"]["iter"] for e in ev} == {0, 1}


def test_interval_helpers():
    u = tlt._union([(5, 7), (0, 2), (1, 3), (6, 9)])
    assert u == [(0, 3), (5, 9)]
    assert tlt._length(u) == 7
    assert tlt._intersect(u, [(2, 6)]) == 2
    bad = tlt.check([{"pid": 0, "tid": 0, "ts": 0.0, "dur": 5.0, "name": "a", "args": {"iter": 0}},
                     {"pid": 0, "tid": 0, "ts": 4.0, "dur": 1.0, "name": "b", "args": {"iter": 0}}])
    assert len(bad) == 1 and "'b' starts before 'a' ends" in bad[0]


@pytest.mark.gpu
def test_timeline_graph_replay_on_gpu(tmp_path):
    """fsdp on RCCL with a HIP graph: the stamps are captured with the
    iteration, every replay re-reads them; the deadline compute tasks last
    their table time on the device clock."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    out = tmp_path / "tl.json"
    p = subprocess.run([os.path.join(BIN, "fsdp"), "tiny_dense_8_bfloat16", "4", "1", DATA, "--backend", "rccl",
                        "--compute", "gemm", "--graph", "-w", "1", "-r", "3", "--quiet", "--time-scale", "4",
                        "--timeline", str(out)], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, DLNB_NO_TORCH="1"))
    assert p.returncode == 0, p.stderr[-2000:]
    _, ev = _events(out)
    assert tlt.check(ev) == []
    comp = [e for e in ev if e["cat"] == "compute"]
    assert len(comp) == 2 * 8 and {e["args"]["iter"] for e in ev} == {1, 2}
    for e in comp:
        want = e["args"]["table_us"] * 4
        assert 0.95 * want <= e["dur"] <= want + 60.0, e
    # replays differ: the second kept iteration starts after the first ends
    t1 = max(e["ts"] + e["dur"] for e in ev if e["args"]["iter"] == 1)
    assert min(e["ts"] for e in ev if e["args"]["iter"] == 2) >= t1


def test_summarize_graph_launch_edges():
    """DLNB_TIMELINE_EDGES=1 (GPU graph replays): the two stamps on the launch stream around the graph split the
    host boundary into submission, graph start, join and completion detection; they are not device work."""
    def x(cat, name, ts, dur, tid=0):
        return {"ph": "X", "pid": 0, "tid": tid, "cat": cat, "name": name, "ts": ts, "dur": dur, "args": {"iter": 1}}
    ev = [x("host", "iteration (host)", 0.0, 1100.0, 9),
          x("edge", "before graph launch", 10.0, 0.0, 8), x("edge", "after graph launch", 1060.0, 0.0, 8),
          x("comm", "all_gather fsdp/unit/0", 30.0, 100.0, 1), x("compute", "compute", 130.0, 900.0, 2),
          x("comm", "reduce_scatter fsdp/unit/0", 1030.0, 25.0, 1)]
    assert tlt.check(ev) == []
    r = tlt.summarize(ev)["0"]["1"]
    assert r["span_ms"] == pytest.approx(1.025) and r["comm_exposed_ms"] == pytest.approx(0.125)
    assert r["launch_ms"] == pytest.approx(0.030) and r["completion_ms"] == pytest.approx(0.045)
    e = r["edges"]
    assert e["submit_ms"] == pytest.approx(0.010) and e["graph_start_ms"] == pytest.approx(0.020)
    assert e["graph_join_ms"] == pytest.approx(0.005) and e["detect_ms"] == pytest.approx(0.040)
