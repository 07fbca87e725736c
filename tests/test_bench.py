"""bench.py's driver contract: the N > 1 launch (torchrun, one process per
rank, native TCP rendezvous through the store file), exactly one JSON line
from rank 0, honest bus bandwidth (null at 1 rank) and the secondary
comm-bound / compute-stretch blocks. CPU backend here; the GPU variant runs
the same file at N = 1 on the box."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "tests", "data")
TINY = ["--model", "tiny_dense_8_bfloat16", "--base-path", DATA, "--c5-model", "tiny_dense_8_bfloat16",
        "--units", "4", "--c5-steps", "3", "--exact-sizes", "4097,30000"]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_lines(out: str):
    return [json.loads(ln) for ln in out.splitlines() if ln.strip().startswith("{")]


@pytest.mark.parametrize("n", [2, 3])
def test_bench_torchrun_cpu(n, tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "2", "--warmup", "1", "--backend", "cpu", "--compute", "sleep",
           "--link-bench", "on", "--link-sizes", "4096,65536", "--timeline-block", "on"] + TINY
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout  # rank 0 only, nothing else on stdout
    o = lines[0]
    assert o["n_gpus"] == n and o["steps"] == 2 and o["warmup"] == 1
    assert o["config"]["parallelism"] == f"fsdp{n}" and o["config"]["sharding_factor"] == n
    assert o["config"]["global_batch"] == 8 * n
    assert o["higher_is_better"] is False and o["scaling"] == "weak"
    assert o["ms_per_step"] == o["value"] > 0
    assert len(o["per_run_ms"]) == 2 and 0 < o["rank_ms"]["min"] <= o["rank_ms"]["max"] and o["rank_ms"]["slowest_rank"] in range(n)
    # per-iteration attribution: the slowest rank's last collective per iteration (no hwmon
    # sensors on the CPU backend)
    si = o["slow_iterations"]
    assert si["last_collective"] == "reduce_scatter" and len(si["last_collective_ms"]) == 2, si
    assert len(si["exposed_ms"]) == 2 and all(x >= 0 for x in si["exposed_ms"]), si
    assert all(x >= 0 for x in si["last_collective_ms"]) and si["sclk_mhz"] is None, si
    assert o["effective_busbw_GBps"]["allgather"] > 0 and o["effective_busbw_GBps"]["reduce_scatter"] > 0
    c5 = o["comm_bound"]
    assert "error" not in c5, c5
    assert c5["strategy"] == f"dp{n}" and c5["transport"] == "link" and c5["allreduce_busbw_GBps"] > 0
    assert c5["floor_ms"] == pytest.approx(6.0) and c5["ms_per_step"] >= c5["floor_ms"] * 0.9
    assert c5["exposed_comm_ms"] is not None
    assert o["rccl_cta_budget"]["lanes"] == 1
    # the multi-rank exactness pass ran before the timed phases, on every rank
    assert o["exact"] == {"cpu": True, "cpu_eager": True}, o.get("exact_detail")
    d = o["exact_detail"]
    assert d["ok"] and d["world_size"] == n and d["failed"] == [] and d["sizes"] == [4097, 30000]
    assert d["rccl_nranks"] == -1 and o["rccl_nranks"] == {}  # no RCCL on the CPU backend
    # the collective micro-benchmark on the job's ranks (RCCL / xgmi on GPUs; the shm backend here)
    lb = o["link_bench"]
    assert lb["elements_per_rank"] == [4096, 65536] and "error" not in lb["cpu"], lb
    for op in ("all_reduce", "all_gather", "reduce_scatter", "all_to_all", "sendrecv"):
        assert lb["cpu"][op]["65536"]["busbw_GBps"] > 0 and lb["cpu"][op]["4096"]["time_us"] > 0
    # the cost model refitted to the measured collective times, predictions redone with it
    # (the CPU backend's link times on a host loaded by parallel test workers can leave no positive fit: the
    # block then says so instead of vanishing)
    mf = o["model_fit"]
    assert mf["backend"] == "cpu", mf
    if "error" in mf:
        assert mf["error"].startswith("no fit"), mf
    else:
        assert mf["eta"] > 0 and mf["alpha_us"] >= 0, mf
        assert mf["predicted_ms"]["headline"] > 0 and mf["predicted_ms"]["comm_bound"] > 0
    # the headline config's device timeline, summarised (every rank, last iteration)
    tl = o["timeline"]
    assert "error" not in tl, tl
    assert tl["ranks"] == n and tl["well_formed"] and 0 <= tl["comm_hidden_frac"] <= 1
    assert tl["ops"]["all_gather"]["count"] == 7 * n and tl["ops"]["reduce_scatter"]["count"] == 4 * n
    assert tl["ops"]["all_gather"]["busbw_GBps"] > 0 and tl["span_ms_max"] > 0
    # rank 0's wall seconds per phase, every phase that ran
    ps = o["phase_seconds"]
    assert set(ps) >= {"exact", "headline", "comm_bound", "timeline", "link_bench", "total"}, ps
    assert ps["total"] >= sum(v for k, v in ps.items() if k != "total") - 0.1


def test_bench_hybrid_blocks_eight_ranks_cpu(tmp_path):
    """The N = 8 driver path with the BASELINE C3 / C4 hybrid blocks (hybrid_3d
    S=2 mb=4 T=4, hybrid_3d_moe S=2 mb=8 EP=4 on tiny models), 8 processes on
    the shared-memory backend."""
    n = 8
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n), "--steps", "1", "--warmup", "0", "--backend", "cpu", "--compute", "sleep",
           "--hybrids", "on", "--c3-model", "tiny_deep_8_bfloat16", "--c3", "2,4,4",
           "--c4-model", "tiny_moe_8_bfloat16", "--c4", "2,8,4", "--exact", "off", "--c5-model", "none"] + TINY[:6]
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    o = lines[0]
    h3, h4 = o["hybrid_3d"], o["hybrid_3d_moe"]
    for h in (h3, h4):
        assert "error" not in h, h
        assert h["ms_per_step"] >= 0.9 * h["floor_ms"] > 0 and h["vs_floor"] > 0.9
        assert h["pp_comm_time_ms"] is not None and h["dp_comm_time_ms"] is not None
    assert h3["params"] == [2, 4, 4] and h3["tp_comm_time_ms"] is not None and h3["busbw_GBps"]["tp_allreduce"] > 0
    assert h4["params"] == [2, 8, 4] and h4["ep_comm_time_ms"] is not None and h4["busbw_GBps"]["ep_alltoall"] > 0
    # the same C4 config with the all-to-alls off the compute stream (--ep-overlap)
    ov = h4["ep_overlap"]
    assert "error" not in ov, ov
    assert ov["ep_overlap"] is True and ov["floor_ms"] == h4["floor_ms"] and ov["ms_per_step"] >= 0.9 * ov["floor_ms"]
    # C4 is timed over 2 iterations by default, both blocks, within the default budget
    assert len(h4["per_run_ms"]) == 2 and len(ov["per_run_ms"]) == 2, (h4, ov)
    # the xGMI cost model's prediction next to every measured block
    for h in (h3, h4, ov):
        assert h["predicted_ms"] >= h["floor_ms"] and h["vs_predicted"] > 0
    assert o["predicted_ms"] > 0
    # GPipe floor (mb + S - 1)(f_mb + b_mb): hybrid_3d f_mb = fwd / S / (mb T)
    assert h3["floor_ms"] == pytest.approx((4 + 1) * (2.0 + 4.0) / 2 / (4 * 4), rel=1e-3)
    assert h4["floor_ms"] == pytest.approx((8 + 1) * (2.0 + 4.0) / 2 / 8, rel=1e-3)
    assert {"hybrid_3d", "hybrid_3d_moe", "hybrid_3d_moe_ep_overlap"} <= set(o["phase_seconds"])


def _torchrun(n, args, tmp_path, env=None, timeout=300):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(n)] + args
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=str(tmp_path),
                       env=dict(os.environ, OMP_NUM_THREADS="1", **(env or {})))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    return lines[0]


def test_bench_wall_budget_survives_a_hung_block_two_ranks(tmp_path):
    """a block that hangs on one rank (DLNB_INJECT_FAULT block=c5: rank 1's comm-bound child
    never finishes) costs at most what the wall budget leaves; the line still prints within the budget, the
    hung block reports its timeout and the blocks that no longer fit are skipped, on every rank alike."""
    budget = 40
    o = _torchrun(2, ["--steps", "2", "--warmup", "1", "--backend", "cpu", "--compute", "sleep",
                      "--wall-budget-s", str(budget)] + TINY, tmp_path,
                  env={"DLNB_INJECT_FAULT": "rank=1,iter=0,mode=hang,block=c5"}, timeout=200)
    assert o["value"] > 0 and o["verified"] == {"cpu": True}
    assert o["phase_seconds"]["total"] <= budget
    assert "timeout" in o["comm_bound"]["error"]
    b = o["budget"]
    assert b["wall_budget_s"] == budget and "c5" in b["timeouts_s"] and "c5g" in b["skipped"]
    assert "skipped" in o["comm_bound"]["geometric_buckets"]


def test_bench_headline_fallback_two_ranks(tmp_path):
    """A headline that fails on its backend at N > 1 (rank 1 throws in its first iteration; rank 0's collective
    times out) is timed again on the fallback backend as a bounded child run of every rank: the line carries a
    value, the fallback's backend and the primary failure, and the blocks after it run (on GPU the fallback is
    the xgmi kernels when the exactness pass proved them exact; here --fallback-backend cpu)."""
    o = _torchrun(2, ["--steps", "2", "--warmup", "1", "--backend", "cpu", "--compute", "sleep",
                      "--fallback-backend", "cpu", "--wall-budget-s", "120"] + TINY, tmp_path,
                  env={"DLNB_INJECT_FAULT": "rank=1,iter=0,mode=throw,block=headline", "DLNB_TIMEOUT": "10"},
                  timeout=300)
    assert o["value"] > 0 and "error" not in o, o.get("error")
    fb = o["headline_fallback"]
    assert fb["backend"] == "cpu" and fb["primary_error"] and "error" not in fb, fb
    assert o["config"]["backend"] == "CPU-SHM" and o["comm_bound"]["ms_per_step"] > 0
    assert "headline_fallback" in o["phase_seconds"] and "headline_fallback" in o["budget"]["timeouts_s"]


def test_bench_wall_budget_hybrids_eight_ranks(tmp_path):
    """The N = 8 path with the hybrid blocks and a hang injected into C3 on rank 5: C3 reports its timeout
    (its limit: --hybrid-timeout), the C4 blocks after it still run (per_run_ms: --c4-runs entries), one
    line within the budget."""
    budget = 75
    o = _torchrun(8, ["--steps", "1", "--warmup", "0", "--backend", "cpu", "--compute", "sleep",
                      "--hybrids", "on", "--c3-model", "tiny_deep_8_bfloat16", "--c3", "2,4,4",
                      "--c4-model", "tiny_moe_8_bfloat16", "--c4", "2,8,4", "--c4-runs", "2", "--exact", "off",
                      "--c5-model", "none", "--wall-budget-s", str(budget), "--hybrid-timeout", "25"] + TINY[:6],
                  tmp_path, env={"DLNB_INJECT_FAULT": "rank=5,iter=0,mode=hang,block=c3"}, timeout=300)
    assert o["phase_seconds"]["total"] <= budget
    assert "timeout" in o["hybrid_3d"]["error"], o["hybrid_3d"]
    h4 = o["hybrid_3d_moe"]
    assert "error" not in h4 and len(h4["per_run_ms"]) == 2 and h4["ms_per_step"] > 0, h4
    ov = h4["ep_overlap"]
    assert ("skipped" in ov) or len(ov["per_run_ms"]) == 2, ov


def test_bench_c3_two_timed_runs_eight_ranks(tmp_path):
    """C3 (hybrid_3d) is timed over 2 iterations by default: per_run_ms has both."""
    o = _torchrun(8, ["--steps", "1", "--warmup", "0", "--backend", "cpu", "--compute", "sleep",
                      "--hybrids", "on", "--c3-model", "tiny_deep_8_bfloat16", "--c3", "2,4,4",
                      "--c4-model", "tiny_moe_8_bfloat16", "--c4", "2,8,4", "--c4-ep-overlap", "off",
                      "--exact", "off", "--c5-model", "none"] + TINY[:6], tmp_path, timeout=300)
    h3 = o["hybrid_3d"]
    assert "error" not in h3 and len(h3["per_run_ms"]) == 2 and all(x > 0 for x in h3["per_run_ms"]), h3
    assert len(o["hybrid_3d_moe"]["per_run_ms"]) == 2


def test_bench_links_before_hybrids_eight_ranks(tmp_path):
    """the link evidence (link_bench, then comm_bound_xgmi on GPUs) runs right after C5 and
    before the hybrids, so a C3 that hangs (rank 5, its limit --hybrid-timeout) and a budget too small for
    C4 after it leave link_bench measured and C4 reported skipped."""
    budget = 60
    o = _torchrun(8, ["--steps", "1", "--warmup", "0", "--backend", "cpu", "--compute", "sleep",
                      "--hybrids", "on", "--c3-model", "tiny_deep_8_bfloat16", "--c3", "2,4,4",
                      "--c4-model", "tiny_moe_8_bfloat16", "--c4", "2,8,4", "--exact", "off",
                      "--c5-model", "none", "--link-bench", "on", "--link-sizes", "4096",
                      "--wall-budget-s", str(budget), "--hybrid-timeout", "30"] + TINY[:6],
                  tmp_path, env={"DLNB_INJECT_FAULT": "rank=5,iter=0,mode=hang,block=c3"}, timeout=300)
    assert o["phase_seconds"]["total"] <= budget
    lb = o["link_bench"]
    assert "error" not in lb["cpu"] and "skipped" not in lb, lb
    order = list(o["phase_seconds"])
    assert order.index("link_bench") < order.index("hybrid_3d"), order
    assert "timeout" in o["hybrid_3d"]["error"], o["hybrid_3d"]
    assert "skipped" in o["hybrid_3d_moe"], o["hybrid_3d_moe"]


def test_bench_unverified_backend_flags_its_blocks(tmp_path):
    """with the shm backend's collectives corrupted (DLNB_COMM_FAULT swaps two peers'
    all-gather blocks on rank 0), the exactness pass fails, the line says verified.cpu = false, and the
    headline and the comm-bound block - timed anyway - carry the error."""
    o = _torchrun(2, ["--steps", "2", "--warmup", "1", "--backend", "cpu", "--compute", "sleep"] + TINY, tmp_path,
                  env={"DLNB_COMM_FAULT": "mode=swap,op=all_gather,rank=0"}, timeout=200)
    assert o["verified"] == {"cpu": False} and o["exact"]["cpu"] is False
    assert "exactness failed" in o["error"] and o["value"] > 0
    assert "exactness failed" in o["comm_bound"]["error"] and o["comm_bound"]["ms_per_step"] > 0


def test_bench_two_nodes_cpu(tmp_path):
    """The multi-node launch (torchrun --nnodes 2, 2 ranks per "node", both on
    127.0.0.1): LOCAL_WORLD_SIZE < WORLD_SIZE, so every phase rendezvouses on
    MASTER_PORT + 1 + phase instead of a store file; one JSON line from
    global rank 0, nothing from node 1."""
    port = _free_port()
    procs = []
    for nr in (0, 1):
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=2", f"--node-rank={nr}", "--nproc-per-node=2",
               "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
               "--gpus", "4", "--steps", "2", "--warmup", "1", "--backend", "cpu", "--compute", "sleep"] + TINY
        procs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      cwd=str(tmp_path), env=dict(os.environ, OMP_NUM_THREADS="1")))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (_, err) in zip(procs, outs):
        assert p.returncode == 0, err[-3000:]
    assert _json_lines(outs[1][0]) == []
    lines = _json_lines(outs[0][0])
    assert len(lines) == 1, outs[0][0]
    o = lines[0]
    assert o["n_gpus"] == 4 and o["config"]["sharding_factor"] == 4 and o["config"]["global_batch"] == 32
    assert o["exact"] == {"cpu": True, "cpu_eager": True} and "error" not in o["comm_bound"]
    assert o["effective_busbw_GBps"]["allgather"] > 0


def test_bench_single_rank_reports_no_bus_bandwidth(tmp_path):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "0",
                        "--backend", "cpu", "--compute", "sleep"] + TINY,
                       capture_output=True, text=True, timeout=120, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1
    o = lines[0]
    assert o["n_gpus"] == 1
    # a 1-rank all-gather / reduce-scatter / all-reduce is a local copy: no link bandwidth
    assert o["effective_busbw_GBps"] == {"allgather": None, "reduce_scatter": None}
    assert o["comm_bound"]["allreduce_busbw_GBps"] is None and o["comm_bound"]["transport"] == "local-copy"


def test_busbw_zero_for_one_rank_in_report(data_dir):
    sys.path.insert(0, ROOT)
    from dlnetbench_amd import engine
    d = engine.run("dp", "tiny_dense_8_bfloat16", 4, base_path=data_dir, backend="cpu", compute="sleep", warmup=0,
                   runs=2, silent=True)
    c = d["ranks"][0]["comm"]["allreduce"]
    assert c["transport"] == "local-copy" and c["busbw_GBps"] == 0.0
    b = d["global"]["dlnb"]["rccl_cta_budget"]
    assert b == {"lanes": 1, "comm_cus": 32, "max_ctas_per_lane": 0, "applies": False, "fits": True}


@pytest.mark.gpu
def test_bench_gpu_single_rank_secondaries(tmp_path):
    """bench.py at N = 1 on the GPU with the tiny model: headline + comm-bound
    block + fixed-work compute stretch, one JSON line."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1"] + TINY,
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    o = lines[0]
    assert o["config"]["backend"] == "RCCL" and o["config"]["hip_graph"] is True
    assert o["effective_busbw_GBps"] == {"allgather": None, "reduce_scatter": None}
    c5 = o["comm_bound"]
    assert "error" not in c5, c5
    assert c5["transport"] == "local-copy" and c5["allreduce_busbw_GBps"] is None
    assert c5["ms_per_step"] >= 0.9 * c5["floor_ms"]
    assert 0.8 < c5["gemm_work"]["compute_stretch"] < 1.5, c5
    assert 0.8 < o["compute_stretch"] < 1.5, o
    assert o["rccl_cta_budget"]["applies"] and o["rccl_cta_budget"]["max_ctas_per_lane"] == 32
    # the bench binds /opt/rocm's HIP and RCCL (torch's bundled copies never load: DLNB_NO_TORCH)
    assert o["runtime"]["librccl"].startswith("/opt/rocm") and o["runtime"]["libamdhip64"].startswith("/opt/rocm")
    # the comm-bound step again with RCCL's own CTA count (no maxCTAs cap)
    u = c5["rccl_default_ctas"]
    assert "error" not in u, u
    assert u["ms_per_step"] >= 0.9 * c5["floor_ms"] and u["allreduce_busbw_GBps"] is None
    # energy: the GPU's power sensor integrated over each step (hundreds of W x the step time)
    assert o["energy_J_per_step"] is None or o["energy_J_per_step"]["per_gpu"] > 0
    # per-iteration attribution: last collective, and (hwmon) sclk within its window and power at the end
    si = o["slow_iterations"]
    assert len(si["last_collective_ms"]) == 2, si
    if si["sclk_mhz"] is not None:
        assert all(0 < lo <= x for lo, x in zip(si["sclk_min_mhz"], si["sclk_mhz"])), si
        assert all(p > 0 for p in si["power_w"]), si


@pytest.mark.gpu
def test_bench_gpu_headline_device_fault_still_prints_the_line(tmp_path):
    """a device-side hang injected into the N = 1 headline (its first gate is never raised,
    DLNB_INJECT_FAULT mode=gate, block=headline) costs only the headline's graph child: it exits at the host's
    timeout, the per-iteration retry - a fresh child, where the fault is not armed - times the step, the line
    carries the graph run's error, and the comm-bound block after it reports a normal value."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    env = dict(os.environ, DLNB_INJECT_FAULT="rank=0,iter=0,mode=gate,block=headline", DLNB_TIMEOUT="5")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1",
                        "--no-c5-ctas-ab", "--c5-bucket-ratio", "0", "--stretch-steps", "0"] + TINY,
                       capture_output=True, text=True, timeout=300, cwd=str(tmp_path), env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    o = lines[0]
    assert "exit 3" in o["headline_graph_error"], o.get("headline_graph_error")
    assert o["value"] > 0 and o["config"]["hip_graph"] is False, o
    c5 = o["comm_bound"]
    assert "error" not in c5 and c5["ms_per_step"] >= 0.9 * c5["floor_ms"], c5
    assert c5["ms_per_step"] <= 1.5 * c5["floor_ms"] + 2.0, c5


@pytest.mark.gpu
def test_bench_torchrun_xgmi_two_ranks_one_gpu(tmp_path):
    """The driver's N > 1 launch on the GPU: torchrun, 2 ranks sharing GPU 0 over the xgmi kernels (RCCL
    refuses two ranks on one device), HIP graph, plus the comm_bound_xgmi child-process secondary."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--backend", "xgmi", "--devices", "0,0",
           "--link-sizes", "1048576"] + TINY
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(tmp_path),
                       env=dict(os.environ, DLNB_XGMI_TIMEOUT_S="60"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    o = lines[0]
    assert o["n_gpus"] == 2 and o["config"]["backend"] == "XGMI" and o["config"]["hip_graph"] is True
    assert o["effective_busbw_GBps"]["allgather"] > 0
    x = o["comm_bound_xgmi"]
    assert "error" not in x, x
    assert x["hip_graph"] is True and x["ms_per_step"] > 0 and x["allreduce_busbw_GBps"] > 0
    assert x["speedup_vs_comm_bound"] > 0 and x["comm_bound_backend"] == "XGMI"
    h = o["headline_xgmi"]
    assert "error" not in h, h
    assert h["ms_per_step"] > 0 and h["effective_busbw_GBps"]["allgather"] > 0
    assert h["busbw_ratio_vs_headline"]["allgather"] > 0 and h["headline_backend"] == "XGMI"
    tl = o["timeline"]  # the headline config's device timeline over the xgmi kernels, HIP graph
    assert "error" not in tl and tl["ranks"] == 2 and tl["well_formed"], tl
    assert tl["ops"]["all_gather"]["busbw_GBps"] > 0
    lb = o["link_bench"]  # staged and zero-copy xgmi; no RCCL with 2 ranks on one GPU
    assert "rccl" not in lb and lb["hip_graph"] is True
    for k in ("xgmi", "xgmi_registered"):
        assert "error" not in lb[k], lb
        assert all(lb[k][op]["1048576"]["busbw_GBps"] > 0 for op in ("all_reduce", "all_gather", "sendrecv"))


@pytest.mark.gpu
def test_bench_headline_fallback_two_ranks_one_gpu(tmp_path):
    """The driver's N > 1 launch with the default backend on a job where RCCL cannot form its communicator
    (2 ranks sharing GPU 0 - what a first cross-device RCCL failure looks like to bench.py): the exactness pass
    proves only the xgmi kernels, so the headline runs as a bounded child on RCCL, fails, and is timed on xgmi;
    the line has a value, names the fallback and keeps the RCCL error (profiles/fallback_r4.md)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--devices", "0,0", "--link-sizes", "1048576",
           "--wall-budget-s", "240"] + TINY
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=400, cwd=str(tmp_path),
                       env=dict(os.environ, DLNB_XGMI_TIMEOUT_S="60"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout
    o = lines[0]
    assert o["value"] > 0 and "error" not in o, o.get("error")
    fb = o["headline_fallback"]
    assert fb["backend"] == "xgmi" and "ncclCommInitRank" in fb["primary_error"] and "error" not in fb, fb
    assert o["config"]["backend"] == "XGMI" and o["verified"] == {"xgmi": True}
    assert o["comm_bound"]["ms_per_step"] > 0 and o["comm_bound"]["backend"] == "XGMI"
    assert o["phase_seconds"]["total"] <= 240
