"""Layouts and message sizes: golden values from SURVEY.md §2.4 / BASELINE.md."""
import json
import os

import pytest

from dlnetbench_amd.parallel import plan as P
from dlnetbench_amd.utils.stats import load_stats


@pytest.fixture(scope="module")
def stats(root):
    return lambda n: load_stats(os.path.join(root, "model_stats", n + ".txt"))


def test_grid_3d_reference_layout():
    # hybrid_3d.cpp:283-300: tp_id = rank % T, stage = (rank/T) % S, dp = rank/(T*S)
    T, S, W = 4, 2, 16
    for r in range(W):
        i, s, d = P.grid_coords(r, T, S)
        assert (i, s, d) == (r % T, (r // T) % S, r // (T * S))
        assert r in P.inner_group(r, T, S) and r in P.pp_group(r, T, S) and r in P.dp_group(r, T, S, W)
        # pp rank == stage id (hybrid_3d.cpp:308)
        assert P.pp_group(r, T, S).index(r) == s
    assert P.inner_group(5, 4, 2) == [4, 5, 6, 7]
    assert P.pp_group(5, 4, 2) == [1, 5]
    assert P.dp_group(5, 4, 2, 16) == [5, 13]


def test_grid_2d_reference_layout():
    # hybrid_2d.cpp:272-282: pp groups are contiguous blocks of S ranks
    assert P.pp_group(5, 1, 4) == [4, 5, 6, 7]
    assert P.dp_group(5, 1, 4, 8) == [1, 5]
    assert P.grid_coords(6, 1, 4)[1] == 2


def test_fsdp_groups():
    unit, rep = P.fsdp_groups(5, 4, 8)
    assert unit == [4, 5, 6, 7] and rep == [1, 5]


def test_c2_llama3_8b_fsdp(stats):
    st = stats("llama3_8b_16_bfloat16")
    sh = P.fsdp_shards(st, 32, 8)
    assert sh[0] == 31368208
    pl = P.plan_fsdp(st, 8, 32, 8)
    ag = [m for m in pl.messages if m.name == "allgather"][0]
    assert ag.wire_bytes == 250945664 * 2
    # per-rank wire bytes: 2 AG passes + 1 RS ~ 42.16 GB
    per_rank = (2 * 32 * 7 + 32 * 7) * sh[0] * 2
    assert per_rank / 1e9 == pytest.approx(42.16, abs=0.01)


def test_c3_llama3_70b_hybrid_3d(stats):
    st = stats("llama3_70b_16_bfloat16")
    pl = P.plan_hybrid(st, 8, "hybrid_3d", 2, 4, 4, layers=80)
    m = {x.name: x for x in pl.messages}
    assert m["pipe_sendrecv"].elements == 268435456
    assert m["tp_allreduce"].elements == 67108864 and m["tp_allreduce"].calls_per_iter == 16
    assert m["dp_allreduce"].elements == 8819213312
    assert pl.params["dp_size"] == 1
    assert pl.compute_per_unit_us["fwd_per_microbatch"] == pytest.approx(254109.35, abs=0.01)


def test_c4_mixtral_hybrid_moe(stats):
    st = stats("mixtral_8x7b_16_bfloat16")
    pl = P.plan_hybrid(st, 8, "hybrid_3d_moe", 2, 16, 4, layers=32)
    m = {x.name: x for x in pl.messages}
    assert m["ep_alltoall"].elements == 67108864
    assert m["ep_alltoall"].calls_per_iter == 1024
    assert m["dp_allreduce"].elements == 6475349088


def test_c5_vit_h_dp(stats):
    st = stats("vit_h_32_float8")
    pl = P.plan_dp(st, 8, 1)
    assert pl.messages[0].elements == 632404480


def test_dp_bucket_remainder(stats):
    st = stats("gpt2_l_16_bfloat16")
    sizes = P._split(st.model_size, 7)
    assert sum(sizes) == st.model_size and max(sizes) - min(sizes) <= 1
    assert sizes[0] >= sizes[-1]


def test_busbw_factors():
    assert P.busbw_factor("allreduce", 8) == pytest.approx(1.75)
    assert P.busbw_factor("allgather", 8) == pytest.approx(0.875)
    assert P.busbw_factor("sendrecv", 2) == 1.0
    assert P.busbw_factor("allreduce", 1) == 0.0


def test_invalid_layouts(stats):
    st = stats("llama3_8b_16_bfloat16")
    with pytest.raises(ValueError):
        P.plan_fsdp(st, 6, 4, 4)
    with pytest.raises(ValueError):
        P.plan_hybrid(st, 8, "hybrid_3d", 3, 4, 2, layers=32)



def test_plan_dp_zero(stats):
    st = stats("llama3_8b_16_bfloat16")
    base = P.plan_dp(st, 8, 10)
    z1 = P.plan_dp(st, 8, 10, zero=1)
    z2 = P.plan_dp(st, 8, 10, zero=2)
    b0 = base.messages[0].elements
    shard = -(-b0 // 8)
    assert [m.op for m in z1.messages] == ["allreduce", "allgather"]
    assert [m.op for m in z2.messages] == ["reduce_scatter", "allgather"]
    assert z2.messages[0].elements == shard and z2.messages[1].wire_bytes == shard * 8 * 2
    # ZeRO-2 moves half the gradient bytes of an all-reduce per rank (busbw factor (n-1)/n vs 2(n-1)/n)
    assert P.busbw_factor("reduce_scatter", 8) * 2 == P.busbw_factor("allreduce", 8)
    assert z2.memory_bytes < z1.memory_bytes


def test_plan_4d_and_cp(stats):
    st = stats("mixtral_8x7b_16_bfloat16")
    p4 = P.plan_hybrid(st, 16, "hybrid_4d", 2, 16, 2, 32, experts=4)
    names = {m.name: m for m in p4.messages}
    assert names["ep_alltoall"].elements == (1 * st.seq_len * 2 * st.hidden) // 4 // 2
    assert names["tp_allreduce"].elements == st.seq_len * st.hidden // 2
    assert names["dp_allreduce"].group_size == 1
    # E = 1, T = 1 4-D plan degenerates to the hybrid_3d_moe message sizes at EP = 1
    moe = {m.name: m for m in P.plan_hybrid(st, 2, "hybrid_3d_moe", 2, 16, 1, 32).messages}
    d4 = {m.name: m for m in P.plan_hybrid(st, 2, "hybrid_4d", 2, 16, 1, 32, experts=1).messages}
    assert d4["ep_alltoall"].elements == moe["ep_alltoall"].elements
    assert d4["dp_allreduce"].elements == moe["dp_allreduce"].elements
    l8 = stats("llama3_8b_16_bfloat16")
    ring = P.plan_cp(l8, 8, 8, 32, 32, 8)
    kv = 2 * 16 * (8192 // 8) * (4096 * 8 // 32)
    assert ring.messages[0].elements == kv and ring.messages[0].calls_per_iter == 32 * 7
    uly = P.plan_cp(l8, 8, 8, 32, 32, 8, algo="ulysses")
    assert uly.messages[0].op == "alltoall" and uly.messages[0].calls_per_iter == 64


@pytest.mark.parametrize("semantics", ["rendezvous", "buffered"])
@pytest.mark.parametrize("sched,V", [("gpipe", 1), ("1f1b", 1), ("interleaved", 2), ("interleaved", 3)])
@pytest.mark.parametrize("S,mb", [(1, 2), (2, 2), (2, 4), (3, 6), (4, 4), (4, 8), (8, 8), (8, 16)])
def test_schedule_model_no_deadlock_and_floor(sched, V, S, mb, semantics):
    """The enqueue order of every pipeline schedule (model of strategy_pipeline.cpp) never deadlocks - with
    RCCL-like rendezvous groups or the xgmi / shared-memory backends' buffered sends - and reaches the
    driver's compute floor when links cost nothing."""
    from dlnetbench_amd.parallel import schedule_sim as sim
    t, stuck = sim.simulate(sim.build(S, mb, V, 1.0, 2.0, sched), semantics)
    assert not stuck
    assert t == pytest.approx(sim.floor(S, mb, V, 1.0, 2.0))


@pytest.mark.parametrize("semantics", ["rendezvous", "buffered"])
@pytest.mark.parametrize("S,mb", [(2, 2), (2, 4), (4, 4), (4, 8), (4, 16), (6, 12), (8, 8), (8, 16), (8, 32), (16, 32)])
def test_dualpipe_model_no_deadlock_and_beats_1f1b(S, mb, semantics):
    """DualPipe's tick order (build_dualpipe in strategy_pipeline.cpp) never deadlocks, reaches its own compute
    floor when links cost nothing, and that floor sits between the bubble-free mb (f + b) and 1F1B's
    (mb + S - 1)(f + b), within 3 (f + b) of the ideal mb (f + b) + (S/2 - 1)(f + b)."""
    from dlnetbench_amd.parallel import schedule_sim as sim
    f, b = 1.0, 2.0
    t, stuck = sim.simulate(sim.build_dualpipe(S, mb, f, b), semantics)
    assert not stuck
    fl = sim.dualpipe_floor(S, mb, f, b)
    assert t == pytest.approx(fl)
    assert mb * (f + b) <= fl < sim.floor(S, mb, 1, f, b)
    if mb >= S:
        assert fl <= (mb + S // 2 - 1) * (f + b) + 3 * (f + b)
    # every rank runs 2 (f + b) per microbatch pair, and at most S + 1 activations are in flight per rank
    ticks = sim.dualpipe_ticks(S, mb)
    for s in range(S):
        live, peak = 0, 0
        for row in ticks:
            if row[s] is not None:
                live += -1 if row[s][2] else 1
                peak = max(peak, live)
        assert live == 0 and peak <= S + 1


# ---- xGMI cost model (dlnetbench_amd/parallel/xgmi_model.py)

def test_xgmi_model_collective_times():
    from dlnetbench_amd.parallel.xgmi_model import LinkModel
    m = LinkModel(link_gbps=100.0, eta=1.0, alpha_us=0.0)
    S = 8e9  # bytes
    assert m.coll_us("allgather", S, 1) == 0.0
    # direct: S / n over each link; ring: (n - 1) / n * S over one link
    assert m.coll_us("allgather", S, 8) == pytest.approx(S / 8 / 1e5)
    assert m.coll_us("allgather", S, 8, "ring") == pytest.approx(S * 7 / 8 / 1e5)
    assert m.coll_us("allreduce", S, 8) == pytest.approx(2 * m.coll_us("reduce_scatter", S, 8))
    assert m.coll_us("sendrecv", S, 2) == pytest.approx(S / 1e5)
    with pytest.raises(ValueError):
        m.coll_us("allgather", S, 16)


def test_xgmi_model_local_hbm_term():
    """Own-kernel data paths: staged (window) kernels move n(3W-1) local bytes per all-gather block, registered
    (zero-copy) ones n(W+1); when that exceeds the link time it bounds the collective."""
    from dlnetbench_amd.parallel.xgmi_model import LinkModel
    S = 8e9  # gathered bytes: 1 GB per rank block at n = 8
    links = LinkModel(link_gbps=1000.0, eta=1.0, alpha_us=0.0)  # fast links: HBM-bound below
    st = LinkModel(link_gbps=1000.0, eta=1.0, alpha_us=0.0, buffers="staged", hbm_gbps=5000.0)
    rg = LinkModel(link_gbps=1000.0, eta=1.0, alpha_us=0.0, buffers="registered", hbm_gbps=5000.0)
    assert links.coll_us("allgather", S, 8) == pytest.approx(1e9 / 1e6)        # 1 GB per link at 1 TB/s
    assert st.local_bytes("allgather", S, 8) == pytest.approx(1e9 * 23)
    assert st.coll_us("allgather", S, 8) == pytest.approx(23e9 / 5e6)          # HBM-bound: 4.6 ms
    assert rg.coll_us("allgather", S, 8) == pytest.approx(9e9 / 5e6)           # 1.8 ms
    assert rg.coll_us("allreduce", 1e9, 8) == pytest.approx(2e9 / 5e6)
    slow = LinkModel(link_gbps=10.0, eta=1.0, alpha_us=0.0, buffers="registered")
    assert slow.coll_us("allgather", S, 8) == pytest.approx(1e9 / 1e4)         # link-bound again


def test_xgmi_model_predictions(root):
    from dlnetbench_amd.parallel import xgmi_model as xm
    st = load_stats(os.path.join(root, "model_stats", "llama3_8b_16_bfloat16.txt"))
    m = xm.LinkModel()
    p1 = xm.predict_fsdp(st, 1, 32, 1, m)
    assert p1["exposed_ms"] == pytest.approx(0.0, abs=1e-9)
    exposed = [xm.predict_fsdp(st, w, 32, w, m)["exposed_ms"] for w in (2, 4, 8)]
    # more links per group -> less exposed time; always a small fraction of the floor
    assert exposed[0] > exposed[1] > exposed[2] > 0
    assert max(exposed) < 0.01 * p1["floor_ms"]
    # a ring over one link per direction exposes more than the direct all-link algorithm
    assert xm.predict_fsdp(st, 8, 32, 8, m, algo="ring")["exposed_ms"] > exposed[2]
    # slower links can only add exposed time
    slow = xm.LinkModel(link_gbps=10.0)
    assert xm.predict_fsdp(st, 8, 32, 8, slow)["exposed_ms"] > exposed[2]
    # dp: iteration >= floor, bucket suggestion is the argmin of the candidates
    vit = load_stats(os.path.join(root, "model_stats", "vit_h_32_float8.txt"))
    best = xm.suggest_buckets(vit, 8, m)
    for nb in (1, 2, 4, 8, 16):
        p = xm.predict_dp(vit, 8, nb, m)
        assert p["iter_ms"] >= p["floor_ms"] - 1e-9
        assert best["iter_ms"] <= p["iter_ms"] + 1e-9


def test_plan_cli_predict(capsys, root):
    from dlnetbench_amd.parallel import plan
    assert plan.main(["fsdp", "llama3_8b_16_bfloat16", "32", "8", "--world", "8", "--base", root, "--predict"]) == 0
    d = json.loads(capsys.readouterr().out)
    by = d["xgmi_prediction"]["by_world"]
    assert set(by) == {"1", "2", "4", "8"} and by["1"]["exposed_ms"] == pytest.approx(0.0, abs=1e-9)


def test_ep_dispatch_counts_match_the_native_run(data_dir):
    """The planner's all-to-allv split equals what the native driver reports."""
    import subprocess
    bin_ = os.path.join(os.path.dirname(data_dir), "..", "build", "bin", "hybrid_3d_moe")
    st = load_stats(os.path.join(data_dir, "model_stats", "tiny_moe_8_bfloat16.txt"))
    pl = P.plan_hybrid(st, 4, "hybrid_3d_moe", 1, 2, 4, 4, ep_imbalance=1.0)
    counts = pl.params["ep_dispatch_elements_per_peer"]
    assert sum(counts) == pl.messages[0].elements * 4 and counts == sorted(counts, reverse=True)
    assert P.ep_dispatch_counts(100, 4, 0.0) == [100] * 4
    if not os.path.exists(bin_):
        pytest.skip("native binaries not built")
    p = subprocess.run([bin_, "tiny_moe_8_bfloat16", "1", "2", "4", data_dir, "--backend", "loopback-cpu", "--ranks",
                        "4", "--ep-imbalance", "1.0", "-w", "0", "-r", "1", "--quiet"], capture_output=True, text=True,
                       timeout=120, env={k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE")})
    from dlnetbench_amd.utils import report
    doc = next(iter(report.parse_output(p.stdout).values()))
    assert doc["global"]["ep_dispatch_bytes_per_peer"] == [c * 2 for c in counts]


@pytest.mark.parametrize("nb,ratio", [(8, 0.7), (8, 1.0), (13, 0.55), (4, 0.9)])
def test_dp_geometric_buckets_match_native(nb, ratio, root):
    """--dp-bucket-ratio: the native driver's bucket sizes (global.bucket_sizes)
    equal plan.dp_bucket_sizes bit for bit, sum to P, shrink geometrically; the
    even policy is the reference's partition."""
    from dlnetbench_amd import engine
    from dlnetbench_amd.parallel.plan import dp_bucket_sizes
    from dlnetbench_amd.utils.stats import load_stats
    st = load_stats(os.path.join(root, "model_stats", "vit_h_32_float8.txt"))
    py = dp_bucket_sizes(st.model_size, nb, ratio)
    assert sum(py) == st.model_size and len(py) == nb
    d = engine.run("dp", "vit_h_32_float8", nb, base_path=root, backend="loopback-cpu", ranks=1, compute="sleep",
                   warmup=0, runs=1, time_scale=0.01, silent=True, dp_bucket_ratio=ratio)
    g = d["global"]
    assert g["bucket_ratio"] == ratio
    if ratio < 1:
        assert g["bucket_policy"] == "geometric" and g["bucket_sizes"] == py
        assert all(a > b for a, b in zip(py[1:-1], py[2:]))
    else:
        assert g["bucket_policy"] == "even" and py == [st.model_size // nb + (i < st.model_size % nb)
                                                      for i in range(nb)]


def test_dp_geometric_tail_shrinks_predicted_n8_step(root):
    """The xGMI model (plan dp --predict): 8 geometric buckets (r = 0.7) take
    the predicted ViT-H N = 8 step from ~7.50 ms (even, the last bucket's
    all-reduce exposed) toward the 7.13 ms floor."""
    from dlnetbench_amd.parallel import xgmi_model as xm
    from dlnetbench_amd.utils.stats import load_stats
    st = load_stats(os.path.join(root, "model_stats", "vit_h_32_float8.txt"))
    lm = xm.LinkModel()
    even = xm.predict_dp(st, 8, 8, lm)["iter_ms"]
    geo = xm.predict_dp(st, 8, 8, lm, ratio=0.7)["iter_ms"]
    assert even == pytest.approx(7.504, abs=0.01)
    assert geo == pytest.approx(7.24, abs=0.01) and geo < even


def test_hybrid_predictions_for_the_baseline_configs(root):
    """plan hybrid_3d / hybrid_3d_moe --predict at N = 8 (the numbers the
    driver's hybrid blocks report as predicted_ms): C3's TP all-reduces and
    stage sends add ~22 ms to the 3.81 s GPipe floor; C4's 1,024 all-to-alls
    on the compute stream add ~1.3 s, and --ep-overlap hides all but ~33 ms."""
    c3 = P.predict("hybrid_3d", "llama3_70b_16_bfloat16", [2, 4, 4], 8, base=root)
    assert c3["floor_ms"] == pytest.approx(3811.64, abs=0.1)
    assert c3["iter_ms"] == pytest.approx(3833.3, abs=1.0)
    c4 = P.predict("hybrid_3d_moe", "mixtral_8x7b_16_bfloat16", [2, 16, 4], 8, base=root)
    c4o = P.predict("hybrid_3d_moe", "mixtral_8x7b_16_bfloat16", [2, 16, 4], 8, base=root, ep_overlap=True)
    assert c4["floor_ms"] == pytest.approx(13557.7, abs=0.1) == c4o["floor_ms"]
    assert c4["iter_ms"] == pytest.approx(14858.8, abs=2.0)
    assert c4o["iter_ms"] == pytest.approx(13590.3, abs=2.0)
    # a ring per collective (a switch fabric's algorithm) costs more than direct all-link collectives
    ring = P.predict("hybrid_3d_moe", "mixtral_8x7b_16_bfloat16", [2, 16, 4], 8, base=root, algo="ring")
    assert ring["iter_ms"] > c4["iter_ms"]


def test_hybrid_prediction_with_free_links_is_the_floor(root):
    """Links of infinite bandwidth and no latency: every schedule's prediction
    is its compute floor (the simulator's critical path), for 1F1B,
    interleaved and DualPipe as well as GPipe."""
    for sched, V in (("gpipe", 1), ("1f1b", 1), ("interleaved", 2), ("dualpipe", 1)):
        r = P.predict("hybrid_2d", "llama3_8b_16_bfloat16", [4, 8], 8, base=root, pp_schedule=sched, pp_virtual=V,
                      link_gbps=1e12, alpha_us=0.0)
        assert r["iter_ms"] == pytest.approx(r["floor_ms"], rel=1e-6), sched


def test_ep_overlap_op_model():
    from dlnetbench_amd.parallel.xgmi_model import _ep_overlap_op_us
    assert _ep_overlap_op_us(100.0, 4, 0.0) == pytest.approx(100.0)
    # all-to-all shorter than a half-slice: hidden except the last one
    assert _ep_overlap_op_us(100.0, 4, 5.0) == pytest.approx(105.0)
    # all-to-all longer than the other half's slice: the lane is the bound
    assert _ep_overlap_op_us(100.0, 4, 50.0) == pytest.approx(12.5 + 8 * 50.0)


def test_link_model_fit_round_trip():
    """fit_link_model recovers eta and alpha from collective times the model
    itself generated at two sizes (the link_bench layout bench.py reports)."""
    from dlnetbench_amd.parallel import xgmi_model as xm
    truth = xm.LinkModel(eta=0.55, alpha_us=25.0)
    for world in (2, 4, 8):
        lb = {}
        for op, kind in xm._FIT_OPS.items():
            for c in (8388608, 67108864):
                nb = c * 2 * (world if kind in ("allgather", "reduce_scatter", "alltoall") else 1)
                lb.setdefault(op, {})[str(c)] = {"time_us": truth.coll_us(kind, nb, world if kind != "sendrecv" else 2)}
        f = xm.fit_link_model(lb, world)
        assert f["eta"] == pytest.approx(0.55, rel=1e-3) and f["alpha_us"] == pytest.approx(25.0, abs=0.05)
        assert set(f["per_op"]) == set(xm._FIT_OPS)
    assert xm.fit_link_model({"all_reduce": {"8": {"time_us": 5.0}}}, 8)["eta"] is None  # one size: no fit



@pytest.mark.parametrize("sched", ["gpipe", "1f1b", "interleaved", "dualpipe"])
def test_hybrid_predictions_every_schedule(root, sched):
    """Every pipeline schedule of hybrid_2d and hybrid_4d simulates to completion with real link times
    (no deadlock in the model) and lands at or above its compute floor."""
    for strat, model, params in (("hybrid_2d", "llama3_8b_16_bfloat16", [4, 8]),
                                 ("hybrid_4d", "mixtral_8x7b_16_bfloat16", [2, 16, 2, 2])):
        r = P.predict(strat, model, params, 8, base=root, pp_schedule=sched, pp_virtual=2)
        assert r["iter_ms"] >= r["floor_ms"] > 0 and r["sendrecv_us"] > 0
