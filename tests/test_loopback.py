"""The loopback backend: N ranks as threads of ONE process on one device.

SURVEY.md §4 asks for every driver at W = 1, 2, 4, 8 "as single-process
multi-rank" (§7.4 H1: RCCL refuses two ranks on one device). The loopback
backend runs the same strategy code, timers and report N-wide inside one
process. These CPU tests use `--backend loopback-cpu`, which puts every rank
thread on the CPU device and makes no HIP call. The GPU variant
(`--backend loopback`, all ranks on one MI355X) runs only in the
`@pytest.mark.gpu` tests of tests/test_gpu_strategies.py.

Checks: exact collectives and P2P (dlnb commtest), every strategy's report at
W = N with the golden key sets of the shared-memory backend, and that a
failing rank thread ends the job instead of leaving the others blocked.
"""
import json
import os
import subprocess
import sys

import pytest

from dlnetbench_amd.utils import report

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin")
DLNB = os.path.join(BIN, "dlnb")
BACKEND = "loopback-cpu"

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_cpu_strategies import DP_GLOBAL, DP_RANK, FSDP_GLOBAL, FSDP_RANK, PP_GLOBAL, PP_RANK  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def binaries():
    if not os.path.exists(DLNB):
        pytest.skip("native binaries not built (run make)")


def _env(extra=None):
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "DLNB_RANK", "DLNB_WORLD_SIZE"):
        env.pop(k, None)
    env.update(extra or {})
    return env


def run(n, prog, *args, timeout=120, env=None):
    p = subprocess.run([os.path.join(BIN, prog), *map(str, args), "--backend", BACKEND, "--ranks", str(n),
                        "--quiet"], capture_output=True, text=True, timeout=timeout, env=_env(env), cwd=ROOT)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-3000:]
    docs = report.parse_output(p.stdout)
    assert len(docs) == 1, p.stdout[-2000:]
    return next(iter(docs.values()))


@pytest.mark.parametrize("w", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("dtype", ["bf16", "fp32", "fp8_e4m3"])
def test_commtest_loopback_exact(w, dtype):
    p = subprocess.run([DLNB, "commtest", "--backend", BACKEND, "--ranks", str(w), "--dtype", dtype, "--sizes",
                        "1,7,100,4097,70001"], capture_output=True, text=True, timeout=120, env=_env(), cwd=ROOT)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0 and lines, p.stdout[-2000:] + p.stderr[-3000:]
    assert lines[0]["ok"] and lines[0]["world_size"] == w and lines[0]["backend"] == "LOOPBACK"


def test_commtest_loopback_bench():
    p = subprocess.run([DLNB, "commtest", "--backend", BACKEND, "--ranks", "4", "--bench", "--sizes", "4096",
                        "--iters", "2", "--warmup", "1"], capture_output=True, text=True, timeout=120, env=_env(),
                       cwd=ROOT)
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert p.returncode == 0, p.stderr[-2000:]
    assert {ln["op"] for ln in lines} == {"all_reduce", "all_gather", "reduce_scatter", "all_to_all", "copy",
                                          "sendrecv"}
    assert all(ln["busbw_GBps"] > 0 for ln in lines if ln["op"] != "copy")


@pytest.mark.parametrize("w", [1, 2, 4, 8])
def test_dp_loopback(w, data_dir):
    d = run(w, "dp", "tiny_dense_8_bfloat16", 5, data_dir, "-w", 1, "-r", 3)
    g = d["global"]
    assert DP_GLOBAL <= set(g) and g["world_size"] == w and g["backend"] == "LOOPBACK"
    assert g["dlnb"]["ranks_on_device"] == w  # every rank thread on the one device
    assert len(d["ranks"]) == w
    for r in d["ranks"]:
        assert DP_RANK <= set(r) and len(r["runtimes"]) == 3


@pytest.mark.parametrize("zero", [1, 2])
def test_dp_zero_loopback(zero, data_dir):
    d = run(4, "dp", "tiny_dense_8_bfloat16", 5, data_dir, "-w", 1, "-r", 2, "--zero", zero)
    assert d["global"]["world_size"] == 4 and len(d["ranks"]) == 4


@pytest.mark.parametrize("w,U,F", [(2, 4, 2), (4, 4, 4), (8, 4, 4)])
def test_fsdp_loopback(w, U, F, data_dir):
    d = run(w, "fsdp", "tiny_dense_8_bfloat16", U, F, data_dir, "-w", 1, "-r", 2)
    g = d["global"]
    assert FSDP_GLOBAL <= set(g) and g["world_size"] == w and g["num_replicas"] == w // F
    for r in d["ranks"]:
        assert FSDP_RANK <= set(r) and len(r["allgather"]) == 2


@pytest.mark.parametrize("sched", ["gpipe", "1f1b"])
def test_hybrid_2d_loopback(sched, data_dir):
    d = run(4, "hybrid_2d", "tiny_dense_8_bfloat16", 2, 4, data_dir, "-w", 1, "-r", 2, "--pp-schedule", sched)
    g = d["global"]
    assert PP_GLOBAL <= set(g) and g["dp_size"] == 2
    assert all(PP_RANK <= set(r) for r in d["ranks"])


@pytest.mark.parametrize("w,S,mb,V", [(2, 2, 4, 2), (4, 4, 4, 2), (4, 4, 8, 3), (8, 4, 8, 2), (6, 2, 4, 4)])
def test_hybrid_2d_interleaved_loopback(w, S, mb, V, data_dir):
    # Groups complete on the host here, so the interleaved enqueue order (a
    # ring through the wrap link) must be free of host-level cycles too.
    d = run(w, "hybrid_2d", "tiny_deep_8_bfloat16", S, mb, data_dir, "-w", 1, "-r", 2, "--pp-schedule",
            "interleaved", "--pp-virtual", V, timeout=60)
    assert d["global"]["num_stages"] == S and len(d["ranks"]) == w


@pytest.mark.parametrize("sched", ["gpipe", "1f1b"])
def test_hybrid_2d_deep_pipeline_loopback(sched, data_dir):
    d = run(8, "hybrid_2d", "tiny_deep_8_bfloat16", 8, 8, data_dir, "-w", 1, "-r", 2, "--pp-schedule", sched,
            timeout=60)
    assert d["global"]["num_stages"] == 8


@pytest.mark.parametrize("prog,model,params,w,extra", [
    ("hybrid_3d", "tiny_dense_8_bfloat16", (2, 4, 2), 8, ()),
    ("hybrid_3d", "tiny_dense_8_bfloat16", (2, 4, 2), 4, ("--sequence-parallel",)),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", (2, 4, 2), 8, ()),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", (2, 4, 2), 4, ("--ep-overlap",)),
    ("hybrid_4d", "tiny_moe_8_bfloat16", (2, 2, 2, 2), 8, ()),
    ("hybrid_cp", "tiny_dense_8_bfloat16", (2,), 4, ()),
    ("hybrid_cp", "tiny_dense_8_bfloat16", (4,), 4, ("--cp-algo", "ulysses")),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", (1, 2, 4), 4, ("--ep-imbalance", "1.0")),
    ("hybrid_4d", "tiny_moe_8_bfloat16", (2, 2, 2, 2), 8, ("--ep-imbalance", "1.5")),
    ("hybrid_2d", "tiny_deep_8_bfloat16", (4, 8), 8, ("--pp-schedule", "dualpipe")),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", (2, 4, 2), 8, ("--pp-schedule", "dualpipe", "--ep-imbalance", "1")),
])
def test_hybrids_loopback(prog, model, params, w, extra, data_dir):
    d = run(w, prog, model, *params, data_dir, "-w", 1, "-r", 2, *extra)
    assert d["global"]["world_size"] == w and len(d["ranks"]) == w


def test_loopback_rank_failure_ends_the_job(data_dir):
    # rank 1 throws at its second iteration; the other rank threads leave
    # their collectives / barriers and the job exits with the rank's error
    p = subprocess.run([os.path.join(BIN, "dp"), "tiny_dense_8_bfloat16", "2", data_dir, "--backend", BACKEND,
                        "--ranks", "3", "--quiet", "-w", "2", "-r", "2"], capture_output=True, text=True,
                       timeout=90, env=_env({"DLNB_INJECT_FAULT": "rank=1,iter=1,mode=throw"}), cwd=ROOT)
    assert p.returncode == 2, p.stderr[-2000:]
    assert "rank 1" in p.stderr and "DLNB_INJECT_FAULT" in p.stderr


def test_loopback_refuses_a_multi_process_launch(data_dir):
    p = subprocess.run([os.path.join(BIN, "dp"), "tiny_dense_8_bfloat16", "2", data_dir, "--backend", BACKEND,
                        "--ranks", "2", "--quiet"], capture_output=True, text=True, timeout=60,
                       env=_env({"WORLD_SIZE": "2", "RANK": "0"}), cwd=ROOT)
    assert p.returncode == 2 and "one process" in p.stderr


_LIBRARY_FAILURE = r"""
import json, os, sys, time
sys.path.insert(0, {root!r})
os.environ["DLNB_NO_TORCH"] = "1"
from dlnetbench_amd import engine, _native
data = {data!r}
os.environ["DLNB_INJECT_FAULT"] = "rank=1,iter=1,mode={mode}"
t0 = time.time()
try:
    engine.run("dp", "tiny_dense_8_bfloat16", 2, base_path=data, backend="loopback-cpu", ranks=3, warmup=1, runs=2,
               compute="sleep", silent=True)
    print("NO ERROR")
except _native.NativeError as e:
    print("RAISED", time.time() - t0, str(e)[:200])
del os.environ["DLNB_INJECT_FAULT"]
# the failed job's abort switch is its own: later runs in this process are unaffected - except that a
# loopback job is refused while a detached rank thread of an earlier one still lives (it holds streams)
try:
    d = engine.run("dp", "tiny_dense_8_bfloat16", 2, base_path=data, backend="loopback-cpu", ranks=3, warmup=1,
                   runs=2, compute="sleep", silent=True)
    print(json.dumps({{"ok": d["global"]["dlnb"]["iteration"]["median_ms"]}}))
except _native.NativeError as e:
    print(json.dumps({{"refused": str(e)[:300]}}))
d = engine.run("dp", "tiny_dense_8_bfloat16", 2, base_path=data, backend="cpu", warmup=1, runs=2, compute="sleep",
               silent=True)
print(json.dumps({{"cpu": d["global"]["dlnb"]["iteration"]["median_ms"]}}))
"""


@pytest.mark.parametrize("mode", ["throw", "hang"])
def test_loopback_failure_in_library_mode_raises(mode, data_dir, root):
    """In-process (Python / ctypes) loopback jobs: a failing rank raises
    NativeError instead of ending the interpreter; a rank thread that never
    leaves its wait (injected hang) is detached after the grace period; the
    job-scoped CPU abort switch leaves later runs in the process intact."""
    env = dict(os.environ, DLNB_STORE_TIMEOUT="3", DLNB_LOOPBACK_ABORT_GRACE_S="1")
    p = subprocess.run([sys.executable, "-c", _LIBRARY_FAILURE.format(root=root, data=data_dir, mode=mode)],
                       capture_output=True, text=True, timeout=120, env=env)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    lines = p.stdout.splitlines()
    assert lines[0].startswith("RAISED"), p.stdout
    cpu = json.loads(lines[2])["cpu"]
    assert cpu >= 0.9 * 6.0  # tiny model: 6 ms of compute per iteration, nothing dropped
    if mode == "hang":
        assert "detached" in lines[0] and float(lines[0].split()[1]) < 30
        # the hung rank thread never exits: no further loopback job in this process
        assert "still has 1 rank threads blocked" in json.loads(lines[1])["refused"]
    else:
        assert json.loads(lines[1])["ok"] >= 0.9 * 6.0
