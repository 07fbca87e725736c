"""Exact collective checks (dlnb commtest) for every backend.

CPU: the shared-memory backend at W = 1..4 in every wire dtype.
GPU: RCCL at W=1, and the xgmi backend's own kernels with 2 and 4 ranks
sharing one MI355X (-d 0,0,..: IPC within a device exercises the same
windows, flags and kernels as across xGMI), with small windows so every
operation is cut into many pieces. Strategies also run end to end on xgmi.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DLNB = os.path.join(ROOT, "build", "bin", "dlnb")


def launch(n, args, env_extra=None, timeout=140):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(env_extra or {})
    cmd = [sys.executable, "-m", "dlnetbench_amd.utils.launch", "-n", str(n), "--timeout", str(timeout)] + args
    return subprocess.run(cmd, capture_output=True, text=True, timeout=timeout + 30, env=env, cwd=ROOT)


def commtest(n, *extra, env_extra=None):
    p = launch(n, [DLNB, "commtest", *extra], env_extra)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-3000:]
    return [json.loads(ln) for ln in lines]


@pytest.mark.parametrize("w", [1, 2, 3, 4])
@pytest.mark.parametrize("dtype", ["bf16", "fp32", "fp16", "fp8_e4m3", "fp8_e5m2"])
def test_cpu_backend_exact(w, dtype):
    out = commtest(w, "--backend", "cpu", "--dtype", dtype, "--sizes", "1,7,100,4097,70001")
    assert out[0]["ok"] and out[0]["world_size"] == w and out[0]["backend"] == "CPU-SHM"


@pytest.mark.parametrize("w,dtype", [(2, "bf16"), (3, "fp32"), (4, "fp8_e4m3")])
def test_cpu_backend_registered_exact(w, dtype):
    """--registered on the shm backend: memfd buffers every member maps, so the
    collectives read and write the members' buffers directly (all-reduce out of
    place and in place, all-gather, reduce-scatter, all-to-all), exactly."""
    out = commtest(w, "--backend", "cpu", "--registered", "--dtype", dtype, "--sizes", "1,7,100,4097,70001")
    assert out[0]["ok"] and out[0]["registered"] is True and out[0]["backend"] == "CPU-SHM"


FAULTS = ["mode=swap,op=all_gather", "mode=swap,op=all_to_all,rank=1", "mode=swap,op=all_reduce,rank=1",
          "mode=swap,op=reduce_scatter,rank=0", "mode=swap,op=recv,rank=1", "mode=skip,op=all_gather",
          "mode=skip,op=reduce_scatter", "mode=skip,op=recv", "mode=skip,op=all_reduce,call=1"]


@pytest.mark.parametrize("dtype", ["bf16", "fp8_e4m3", "fp8_e5m2"])
@pytest.mark.parametrize("fault", FAULTS)
def test_exactness_check_catches_injected_faults(fault, dtype):
    """Mutation check of the exactness pass: a peer / offset misroute (swap two
    parts of an op's output) or an op that never ran (skip: its output keeps stale data) fails the check
    in every dtype, fp8 included (DLNB_COMM_FAULT, csrc/src/comm_fault.cpp)."""
    p = launch(2, [DLNB, "commtest", "--backend", "cpu", "--dtype", dtype, "--sizes", "64,4097"],
               {"DLNB_COMM_FAULT": fault}, timeout=100)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode != 0 and lines and not lines[0]["ok"] and lines[0]["failures"] > 0, p.stdout + p.stderr[-2000:]


@pytest.mark.parametrize("fault", ["mode=swap,op=all_gather", "mode=swap,op=all_to_all,rank=1",
                                   "mode=swap,op=recv,rank=1"])
def test_legacy_fp8_pattern_missed_misroutes(fault):
    """Why the patterns changed: with round 3's fp8 pattern (1.0 for every rank and element) the same
    misroutes pass unnoticed; the hashed patterns above catch them."""
    p = launch(2, [DLNB, "commtest", "--backend", "cpu", "--dtype", "fp8_e4m3", "--sizes", "64,4097"],
               {"DLNB_COMM_FAULT": fault, "DLNB_COMMTEST_LEGACY_PATTERN": "1"}, timeout=100)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines[0]["ok"], p.stdout + p.stderr[-2000:]


def test_suite_reports_injected_fault_per_combination(tmp_path):
    """--suite (bench.py's exactness pass) on the CPU backend: the faulty combination is reported failed
    and the verdict is all-reduced (every rank writes the same report)."""
    out = tmp_path / "suite.json"
    p = launch(2, [DLNB, "commtest", "--suite", "--backends", "cpu", "--dtypes", "bf16,fp8_e4m3",
                   "--sizes", "4097,30000", "--json", str(out)], {"DLNB_COMM_FAULT": "mode=swap,op=all_gather"},
               timeout=100)
    d = json.loads(out.read_text())
    assert p.returncode != 0 and d["ok"] is False and d["exact"]["cpu"] is False
    assert {(r["dtype"], r["ok"]) for r in d["results"]} == {("bf16", False), ("fp8_e4m3", False)}


def test_suite_eight_ranks_time_cpu(tmp_path):
    """The exactness pass at N = 8 with bench.py's sizes stays within its time budget (here the CPU
    backend on this container: 8 processes, every op poisoned and checked)."""
    out = tmp_path / "suite.json"
    p = launch(8, [DLNB, "commtest", "--suite", "--backends", "cpu", "--dtypes", "bf16,fp8_e4m3",
                   "--sizes", "4097,300000,2097157", "--json", str(out)], timeout=200)
    d = json.loads(out.read_text())
    assert p.returncode == 0 and d["ok"] and d["world_size"] == 8, p.stderr[-2000:]
    assert d["seconds"] < 20, d["seconds"]


def test_cpu_registered_falls_back_when_a_peer_cannot_map():
    """a rank that cannot open a peer's buffer (separate PID namespace, hidepid /proc) no longer
    fails the run: every member marks that registration unusable and the ops take the staged path, exactly."""
    p = launch(2, [DLNB, "commtest", "--backend", "cpu", "--registered", "--dtype", "bf16", "--sizes", "7,4097"],
               {"DLNB_SHM_NO_PEER_MAP": "1"}, timeout=100)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines[0]["ok"], p.stdout + p.stderr[-2000:]
    assert "staged (copy) path" in p.stderr


def test_cpu_backend_bench_lines():
    out = commtest(2, "--backend", "cpu", "--bench", "--sizes", "4096,65536", "--iters", "2", "--warmup", "1")
    ops = {(o["op"], o["count"]) for o in out}
    assert len(ops) == 12  # 4 collectives + ring send/recv + the local copy roofline, 2 sizes
    for o in out:
        assert o["time_us"] > 0 and (o["busbw_GBps"] > 0 or o["op"] == "copy")


def test_commtest_usage():
    p = subprocess.run([DLNB, "commtest", "--help"], capture_output=True, text=True)
    assert p.returncode == 0 and "commtest" in p.stdout
    p = subprocess.run([DLNB, "commtest", "--bogus"], capture_output=True, text=True)
    assert p.returncode == 2


# ----------------------------------------------------------------- GPU


def _need_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


SMALL_WINDOWS = {"DLNB_XGMI_REGION_MB": "1", "DLNB_XGMI_P2P_MB": "1", "DLNB_XGMI_TIMEOUT_S": "60"}


@pytest.mark.gpu
def test_rccl_single_rank_exact():
    _need_gpu()
    out = commtest(1, "--backend", "rccl")
    assert out[0]["ok"] and out[0]["backend"] == "RCCL"


@pytest.mark.gpu
# (2 ranks, bf16 and fp8 at default windows: test_xgmi_exactness_suite_two_ranks_one_gpu)
@pytest.mark.parametrize("w,dtype", [(2, "bf16"), (2, "fp32"), (4, "fp16"), (3, "bf16")])
def test_xgmi_kernels_exact(w, dtype):
    _need_gpu()
    devs = ",".join(["0"] * w)
    sizes = "1,7,100,4097,65536,300007,1048583"
    out = commtest(w, "--backend", "xgmi", "-d", devs, "--dtype", dtype, "--sizes", sizes, env_extra=SMALL_WINDOWS)
    assert out[0]["ok"] and out[0]["backend"] == "XGMI", out


@pytest.mark.gpu
@pytest.mark.parametrize("w,dtype", [(4, "bf16"), (3, "fp32")])
def test_xgmi_graph_replay_exact(w, dtype):
    """The collectives and a ring send/recv captured into one HIP graph and replayed 3 times with new
    inputs: the kernels take their epochs / message numbers from device counters, so every replay must
    synchronise afresh (a repeated epoch would let a rank read a peer's previous data)."""
    _need_gpu()
    devs = ",".join(["0"] * w)
    out = commtest(w, "--backend", "xgmi", "-d", devs, "--dtype", dtype, "--graph", "--sizes", "1,100,4097,300007",
                   env_extra=SMALL_WINDOWS)
    assert out[0]["ok"] and out[0]["graph"] is True, out


@pytest.mark.gpu
@pytest.mark.parametrize("w,dtype,graph", [(4, "bf16", False), (3, "fp32", False), (4, "fp16", True)])
def test_xgmi_registered_zero_copy_exact(w, dtype, graph):
    """--registered: peer-memory buffers registered with the communicator, so all-gather writes straight
    into every rank's receive buffer, reduce-scatter reads straight out of every rank's send buffer and the
    all-reduce (16-B multiples above the one-shot range) does both - no window staging. Exact, eager and
    graph-replayed; the odd sizes take the staged paths on the same buffers."""
    _need_gpu()
    devs = ",".join(["0"] * w)
    extra = ["--graph"] if graph else []
    out = commtest(w, "--backend", "xgmi", "-d", devs, "--dtype", dtype, "--registered", *extra,
                   "--sizes", "1,100,4097,65536,300000,1048583,2097152", env_extra=SMALL_WINDOWS)
    assert out[0]["ok"] and out[0]["registered"] is True, out


@pytest.mark.gpu
def test_rccl_graph_replay_exact():
    _need_gpu()
    out = commtest(1, "--backend", "rccl", "--graph", "--sizes", "1,4097")
    assert out[0]["ok"] and out[0]["graph"] is True


@pytest.mark.gpu
@pytest.mark.parametrize("graph", [False, True])
def test_mixed_backend_single_rank_exact(graph):
    """--backend mixed (size-based RCCL / xgmi dispatch) at W = 1, the only rank count RCCL allows on one GPU:
    every op and size routes through the dispatcher and stays exact."""
    _need_gpu()
    extra = ["--graph"] if graph else []
    out = commtest(1, "--backend", "mixed", "--sizes", "1,4097,1048583", *extra, env_extra={"DLNB_MIXED_XGMI_MAX_KB": "64"})
    assert out[0]["ok"] and out[0]["backend"] == "RCCL", out  # one rank: no xgmi side


MIXED_ALL_XGMI = {"DLNB_MIXED_XGMI_MAX_KB": str(8 << 20), "DLNB_XGMI_TIMEOUT_S": "60"}


@pytest.mark.gpu
def test_mixed_backend_two_ranks_xgmi_side():
    """--backend mixed with 2 ranks on one GPU: with a threshold above every message the groups need no RCCL
    side (RCCL refuses two ranks on one device), so the dispatcher's routing of collectives and grouped
    point-to-point runs end to end through its xgmi side, exactly."""
    _need_gpu()
    out = commtest(2, "--backend", "mixed", "-d", "0,0", "--sizes", "1,4097,300000", env_extra=MIXED_ALL_XGMI)
    assert out[0]["ok"] and out[0]["backend"] == "XGMI", out


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,model,params,extra,w", [
    ("fsdp", "tiny_dense_8_bfloat16", ["4", "2"], ["--graph"], 2),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", ["1", "2", "2"], [], 2)])
def test_strategies_on_mixed_two_ranks(strategy, model, params, extra, w, tmp_path):
    _need_gpu()
    out = tmp_path / "r.json"
    data = os.path.join(ROOT, "tests", "data")
    args = [os.path.join(ROOT, "build", "bin", strategy), model, *params, data, *extra, "-w", "1", "-r", "2",
            "--backend", "mixed", "-d", ",".join(["0"] * w), "--compute", "spin", "--quiet", "--json", str(out)]
    p = launch(w, args, MIXED_ALL_XGMI)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    d = json.loads(out.read_text())
    # the reported group: fsdp's unit group (2 ranks: xgmi side); hybrid_3d_moe's DP group has 1 rank here
    # (RCCL at one rank) while its 2-rank EP group runs on the xgmi side
    assert d["global"]["backend"] == ("XGMI" if strategy == "fsdp" else "RCCL") and len(d["ranks"]) == w


def test_mixed_backend_needs_gpu():
    p = subprocess.run([DLNB, "commtest", "--backend", "mixed"], capture_output=True, text=True,
                       env=dict(os.environ, HIP_VISIBLE_DEVICES="-1"))
    assert p.returncode != 0 and "no GPU" in p.stderr, p.stderr[-500:]


@pytest.mark.gpu
def test_xgmi_default_windows_large_message():
    _need_gpu()
    out = commtest(2, "--backend", "xgmi", "-d", "0,0", "--sizes", "33554441", env_extra={"DLNB_XGMI_TIMEOUT_S": "60"})
    assert out[0]["ok"]


@pytest.mark.gpu
def test_xgmi_bench_runs():
    _need_gpu()
    out = commtest(2, "--backend", "xgmi", "-d", "0,0", "--bench", "--sizes", "65536,4194304", "--iters", "5",
                   "--warmup", "2", env_extra={"DLNB_XGMI_TIMEOUT_S": "60"})
    assert len(out) == 12 and all(o["busbw_GBps"] > 0 for o in out if o["op"] != "copy")


XGMI_STRATS = [  # strategy, model, positional args, extra flags, ranks
    # (2-rank dp / fsdp / hybrid_2d: the graph-replayed, mixed-backend and torchrun bench tests)
    ("dp", "tiny_dense_8_bfloat16", ["4"], [], 8),
    ("fsdp", "tiny_dense_8_bfloat16", ["4", "2"], [], 4),
    ("fsdp", "tiny_dense_8_bfloat16", ["4", "8"], [], 8),
    ("hybrid_2d", "tiny_dense_8_bfloat16", ["2", "4"], ["--pp-schedule", "1f1b"], 4),  # DP 2 x PP 2
    ("hybrid_3d", "tiny_dense_8_bfloat16", ["2", "4", "2"], ["--pp-schedule", "1f1b"], 8),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", ["2", "4", "2"], ["--pp-schedule", "1f1b", "--ep-overlap"], 4),
    ("dp", "tiny_dense_8_bfloat16", ["4"], ["--zero", "2"], 4),
    ("hybrid_cp", "tiny_dense_8_bfloat16", ["2"], [], 4),
    ("hybrid_cp", "tiny_dense_8_bfloat16", ["4"], ["--cp-algo", "ulysses"], 4),
    ("hybrid_4d", "tiny_moe_8_bfloat16", ["2", "2", "2", "2"], ["--pp-schedule", "1f1b"], 8),
    ("hybrid_3d", "tiny_dense_8_bfloat16", ["2", "2", "2"], ["--sequence-parallel"], 4),
    ("hybrid_2d", "tiny_deep_8_bfloat16", ["2", "4"], ["--pp-schedule", "interleaved"], 2),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", ["1", "2", "2"], ["--ep-imbalance", "1.0"], 2),
    ("hybrid_2d", "tiny_deep_8_bfloat16", ["2", "4"], ["--pp-schedule", "dualpipe"], 2),
]


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,model,params,extra,w", XGMI_STRATS)
def test_strategies_on_xgmi(strategy, model, params, extra, w, tmp_path):
    """Up to 8 ranks (a node's worth) sharing one MI355X through the xgmi backend."""
    _need_gpu()
    out = tmp_path / "r.json"
    data = os.path.join(ROOT, "tests", "data")
    args = [os.path.join(ROOT, "build", "bin", strategy), model, *params, data, *extra, "-w", "1", "-r", "2",
            "--backend", "xgmi", "-d", ",".join(["0"] * w), "--compute", "sleep", "--quiet", "--json", str(out)]
    p = launch(w, args, {"DLNB_XGMI_TIMEOUT_S": "60"})
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["global"]["backend"] == "XGMI" and len(d["ranks"]) == w


XGMI_GRAPH_STRATS = [
    ("dp", "tiny_dense_8_bfloat16", ["4"], [], 2),
    ("fsdp", "tiny_dense_8_bfloat16", ["4", "4"], [], 4),
    ("hybrid_2d", "tiny_dense_8_bfloat16", ["2", "4"], ["--pp-schedule", "1f1b"], 2),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", ["1", "2", "2"], [], 2),  # captured EP all-to-alls
]


@pytest.mark.gpu
@pytest.mark.parametrize("strategy,model,params,extra,w", XGMI_GRAPH_STRATS)
def test_strategies_on_xgmi_graph(strategy, model, params, extra, w, tmp_path):
    """One captured iteration replayed (--graph) over the xgmi kernels, ranks sharing one MI355X."""
    _need_gpu()
    out = tmp_path / "r.json"
    data = os.path.join(ROOT, "tests", "data")
    args = [os.path.join(ROOT, "build", "bin", strategy), model, *params, data, *extra, "-w", "1", "-r", "3",
            "--backend", "xgmi", "-d", ",".join(["0"] * w), "--compute", "spin", "--graph", "--quiet",
            "--json", str(out)]
    p = launch(w, args, {"DLNB_XGMI_TIMEOUT_S": "60"})
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    d = json.loads(out.read_text())
    assert d["global"]["backend"] == "XGMI" and d["global"]["dlnb"]["graph"] > 0
    for r in d["ranks"]:
        assert not r.get("async_error"), r


@pytest.mark.gpu
def test_interleaved_shrinks_the_bubble_on_gpu(tmp_path):
    """2 stages sharing one MI355X (xgmi P2P), idle-wait compute 20x the tiny tables: interleaved 1F1B with
    V = 4 finishes an iteration faster than 1F1B (bubble (S-1)/V). Two ranks only: with 4 processes x 4 busy
    streams on one GPU the hardware queues are oversubscribed and time-sliced, and P2P waits then resolve at
    time-slice granularity (profiles/interleaved_xgmi_r1.md)."""
    _need_gpu()
    data = os.path.join(ROOT, "tests", "data")
    med = {}
    for name, extra in (("1f1b", ["--pp-schedule", "1f1b"]),
                        ("il", ["--pp-schedule", "interleaved", "--pp-virtual", "4"])):
        out = tmp_path / f"{name}.json"
        args = [os.path.join(ROOT, "build", "bin", "hybrid_2d"), "tiny_deep_8_bfloat16", "2", "2", data, *extra,
                "-w", "1", "-r", "3", "--backend", "xgmi", "-d", "0,0", "--compute", "sleep", "--time-scale", "20",
                "--quiet", "--json", str(out)]
        p = launch(2, args, {"DLNB_XGMI_TIMEOUT_S": "60"})
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
        it = json.loads(out.read_text())["global"]["dlnb"]["iteration"]
        med[name] = (it["median_ms"], it["compute_floor_ms"])
    assert med["il"][0] < med["1f1b"][0], med
    assert med["il"][0] >= 0.98 * med["il"][1], med


@pytest.mark.gpu
@pytest.mark.parametrize("release", ["vmcnt", "system"])
def test_xgmi_exactness_suite_two_ranks_one_gpu(release):
    """bench.py's multi-GPU exactness pass (commtest --suite) over the xgmi
    kernels with 2 ranks sharing the GPU: staged, registered (zero-copy),
    graph-replayed and registered + replayed, bf16 and fp8, 3 sizes, in both
    release modes of the uncached windows."""
    _need_gpu()
    out = commtest(2, "--suite", "--backends", "xgmi", "-d", "0,0", "--dtypes", "bf16,fp8_e4m3",
                   env_extra={"DLNB_XGMI_RELEASE": release, "DLNB_XGMI_TIMEOUT_S": "30"})
    s = out[0]
    assert s["commtest"] == "suite" and s["world_size"] == 2
    assert s["ok"] and s["exact"]["xgmi"] is True and s["xgmi_release"] == release, s
    for m in ("staged", "registered", "graph", "registered_graph"):
        assert s["exact"]["xgmi_" + m] is True
    assert len(s["results"]) == 8 and all(r["release"] == release for r in s["results"])
    assert s["seconds"] < 60


@pytest.mark.gpu
def test_rccl_exactness_suite_single_rank():
    """The suite's RCCL half at 1 rank (RCCL refuses 2 ranks on one GPU):
    eager + graph, bf16 + fp8, and ncclCommCount reported."""
    _need_gpu()
    s = commtest(1, "--suite", "--backends", "rccl", "--dtypes", "bf16,fp8_e4m3")[0]
    assert s["ok"] and s["exact"] == {"rccl": True, "rccl_eager": True, "rccl_graph": True}, s
    assert s["rccl_nranks"] == 1 and s["runtime"]["librccl"].startswith("/opt/rocm")


@pytest.mark.gpu
@pytest.mark.parametrize("fault", ["mode=swap,op=all_gather", "mode=skip,op=all_to_all", "mode=swap,op=recv,rank=0"])
@pytest.mark.parametrize("dtype", ["bf16", "fp8_e4m3"])
def test_xgmi_graph_check_catches_injected_faults(fault, dtype):
    """The mutation check in HIP-graph mode on the GPU (xgmi kernels, 2 ranks sharing the GPU): a
    misroute captured into the graph, or an op missing from it (its output stays poisoned), fails the
    replayed check in bf16 and in fp8."""
    _need_gpu()
    p = launch(2, [DLNB, "commtest", "--backend", "xgmi", "-d", "0,0", "--graph", "--dtype", dtype,
                   "--sizes", "4097,300000"], dict(SMALL_WINDOWS, DLNB_COMM_FAULT=fault), timeout=100)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode != 0 and lines and not lines[0]["ok"] and lines[0]["graph"], p.stdout + p.stderr[-2000:]
