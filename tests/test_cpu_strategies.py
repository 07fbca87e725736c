"""Every strategy as a multi-process job on the CPU backend (shared memory),
driven through the real CLI binaries and the launcher.

This is the reference's "mpi_cpu" plumbing configuration (README.md:96,
BASELINE.json config 1) made testable: W = 1, 2, 4, 8 ranks, golden report
keys, timer counts, and timing sanity (an iteration can not
be shorter than its compute).
"""
import os
import subprocess

import pytest

from dlnetbench_amd.utils import launch, report

BIN = None


@pytest.fixture(scope="module", autouse=True)
def binaries(root):
    global BIN
    BIN = os.path.join(root, "build", "bin")
    if not os.path.exists(os.path.join(BIN, "dp")):
        pytest.skip("native binaries not built (run make)")


def run(n, prog, *args, timeout=120):
    code, outs = launch.launch(n, [os.path.join(BIN, prog), *map(str, args), "--quiet"], timeout=timeout,
                               capture=True)
    text = "".join(o or "" for o in outs)
    assert code == 0, text[-3000:]
    docs = report.parse_output(outs[0])
    assert len(docs) == 1, outs[0][-2000:]
    return next(iter(docs.values()))


DP_GLOBAL = {"model_name", "num_buckets", "local_batch_size", "world_size", "fwd_rt_whole_model",
             "bwd_rt_per_bucket", "total_model_size_params", "msg_size_avg_bytes", "msg_size_std_bytes",
             "device", "backend"}
DP_RANK = {"runtimes", "barrier_time", "hostname"}
FSDP_GLOBAL = {"model_size_bytes", "model_name", "world_size", "num_units", "sharding_factor", "num_replicas",
               "local_batch_size", "device", "backend", "fwd_time_per_unit_us", "bwd_time_per_unit_us",
               "allgather_msg_size_bytes", "reducescatter_msg_size_bytes"}
FSDP_RANK = {"runtime", "allgather", "allgather_wait_fwd", "allgather_wait_bwd", "reduce_scatter", "barrier",
             "hostname", "rank"}
PP_GLOBAL = {"model_name", "num_stages", "num_microbatches", "samples_per_microbatch", "local_batch_size",
             "global_batch_size", "world_size", "dp_size", "fwd_rt_per_microbatch", "bwd_rt_per_microbatch",
             "total_model_size_params", "pipe_msg_size_bytes", "dp_allreduce_size_bytes", "device", "backend"}
PP_RANK = {"runtimes", "pp_comm_time", "dp_comm_time", "hostname", "stage_id"}


@pytest.mark.parametrize("w", [1, 2, 4, 8])
def test_dp(w, data_dir):
    d = run(w, "dp", "tiny_dense_8_bfloat16", 5, data_dir, "-w", 1, "-r", 3)
    g = d["global"]
    assert DP_GLOBAL <= set(g) and g["world_size"] == w and g["backend"] == "CPU-SHM"
    assert g["num_buckets"] == 5 and g["total_model_size_params"] == 1000003
    # 1000003 / 5 -> buckets of 200001 (x3) and 200000 (x2): bf16 bytes
    assert g["msg_size_avg_bytes"] == pytest.approx(200000.6 * 2)
    assert len(d["ranks"]) == w
    for r in d["ranks"]:
        assert DP_RANK <= set(r)
        assert len(r["runtimes"]) == 3 and len(r["barrier_time"]) == 3 and len(r["allreduce_time"]) == 15
        for rt in r["runtimes"]:
            assert rt >= 0.006 * 0.98  # fwd + bwd = 6 ms of compute
    assert d["global"]["dlnb"]["iteration"]["median_ms"] >= 6.0 * 0.98


@pytest.mark.parametrize("w,zero", [(1, 1), (2, 1), (2, 2), (4, 2), (3, 2), (8, 1), (8, 2)])
def test_dp_zero(w, zero, data_dir):
    """ZeRO-1/2 (extension): sharded optimizer + parameter all-gather, reduce-scatter for stage 2."""
    d = run(w, "dp", "tiny_dense_8_bfloat16", 5, data_dir, "-w", 1, "-r", 2, "--zero", zero)
    g = d["global"]
    assert DP_GLOBAL <= set(g) and g["zero_stage"] == zero
    shard = -(-200001 // w)  # largest bucket 200001 elements, padded to w shards
    assert g["shard_size_params"] == shard
    assert g["param_allgather_msg_size_bytes"] == shard * w * 2
    for r in d["ranks"]:
        assert len(r["runtimes"]) == 2 and len(r["param_allgather_time"]) == 10
        assert len(r["param_allgather_exposed"]) == 2
        key = "reduce_scatter_time" if zero == 2 else "allreduce_time"
        assert len(r[key]) == 10
        other = "allreduce_time" if zero == 2 else "reduce_scatter_time"
        assert len(r[other]) == 0
        kinds = set(r["comm"])
        assert "param_allgather" in kinds and ("reduce_scatter" if zero == 2 else "allreduce") in kinds
        for rt in r["runtimes"]:
            assert rt >= 0.006 * 0.98


def test_dp_zero_rejected_elsewhere(data_dir):
    code, outs = launch.launch(1, [os.path.join(BIN, "fsdp"), "tiny_dense_8_bfloat16", "4", "1", data_dir, "--zero", "1"],
                               timeout=60, capture=True)
    assert code != 0 and "--zero applies to dp" in "".join(o or "" for o in outs)


@pytest.mark.parametrize("w,F", [(2, 2), (4, 2), (4, 4), (8, 8), (8, 4)])
def test_fsdp(w, F, data_dir):
    U = 4
    d = run(w, "fsdp", "tiny_dense_8_bfloat16", U, F, data_dir, "-w", 1, "-r", 2)
    g = d["global"]
    assert FSDP_GLOBAL <= set(g)
    assert g["num_replicas"] == w // F and g["sharding_factor"] == F
    shard = -(-(1000003 // U + 1) // F)  # unit 0 gets the remainder element
    assert g["reducescatter_msg_size_bytes"] == shard * 2
    assert g["allgather_msg_size_bytes"] == shard * F * 2
    if w // F > 1:
        assert "allreduce_msg_size_bytes" in g
    for r in d["ranks"]:
        assert FSDP_RANK <= set(r)
        runs = 2
        assert len(r["runtime"]) == runs
        assert len(r["allgather"]) == runs
        assert len(r["allgather_wait_fwd"]) == runs * (U - 1)
        assert len(r["allgather_wait_bwd"]) == runs * (U - 1)
        assert len(r["reduce_scatter"]) == runs * U
        assert len(r["allreduce_time"]) == (runs * U if w // F > 1 else 0)
        assert min(r["runtime"]) >= 0.006 * 0.98


@pytest.mark.parametrize("lanes", ["single", "split"])
def test_fsdp_comm_lanes(lanes, data_dir):
    d = run(4, "fsdp", "tiny_dense_8_bfloat16", 4, 2, data_dir, "-w", 1, "-r", 2, "--comm-lanes", lanes)
    assert d["global"]["comm_lanes"] == lanes
    for r in d["ranks"]:
        assert len(r["reduce_scatter"]) == 2 * 4 and len(r["allreduce_time"]) == 2 * 4


def test_fsdp_reference_schedule(data_dir):
    d = run(2, "fsdp", "tiny_dense_8_bfloat16", 4, 2, data_dir, "-w", 1, "-r", 2, "--schedule", "reference")
    assert d["global"]["dlnb"]["schedule"] == "reference"


@pytest.mark.parametrize("w,S,mb", [(1, 1, 2), (2, 2, 4), (4, 4, 8), (4, 2, 2), (8, 4, 8)])
def test_hybrid_2d(w, S, mb, data_dir):
    d = run(w, "hybrid_2d", "tiny_dense_8_bfloat16", S, mb, data_dir, "-w", 1, "-r", 2)
    g = d["global"]
    assert PP_GLOBAL <= set(g)
    assert g["dp_size"] == w // S and g["samples_per_microbatch"] == 8 // mb
    assert g["pipe_msg_size_bytes"] == 64 * 128 * (8 // mb) * 2
    assert g["dp_allreduce_size_bytes"] == (1000003 // S) * 2
    stages = sorted(r["stage_id"] for r in d["ranks"])
    assert stages == sorted([r % S for r in range(w)])
    for r in d["ranks"]:
        assert PP_RANK <= set(r)
        assert len(r["pp_comm_time"]) == 2 * mb * 2  # fwd + bwd entries per microbatch, 2 runs
        assert len(r["dp_comm_time"]) == 2
    # GPipe: (mb + S - 1) microbatch slots of (fwd + bwd) per stage
    per_mb = 6.0 / S / mb
    assert g["dlnb"]["iteration"]["median_ms"] >= 0.95 * (mb + S - 1) * per_mb


@pytest.mark.parametrize("w,S,mb", [(2, 2, 4), (4, 4, 8), (4, 4, 2), (4, 2, 1), (2, 2, 8)])
def test_hybrid_2d_1f1b(w, S, mb, data_dir):
    d = run(w, "hybrid_2d", "tiny_dense_8_bfloat16", S, mb, data_dir, "-w", 1, "-r", 2, "--pp-schedule", "1f1b")
    g = d["global"]
    assert g["pp_schedule"] == "1f1b"
    for r in d["ranks"]:
        assert len(r["pp_comm_time"]) == 2 * mb * 2
        assert len(r["dp_comm_time"]) == 2
    # same bubble as GPipe: (mb + S - 1) slots of (fwd + bwd) per microbatch
    per_mb = 6.0 / S / mb
    assert g["dlnb"]["iteration"]["median_ms"] >= 0.95 * (mb + S - 1) * per_mb


@pytest.mark.parametrize("prog,model,params,w", [("hybrid_3d", "tiny_dense_8_bfloat16", (2, 4, 2), 8),
                                                 ("hybrid_3d_moe", "tiny_moe_8_bfloat16", (2, 4, 2), 4)])
def test_hybrid_3d_1f1b(prog, model, params, w, data_dir):
    d = run(w, prog, model, *params, data_dir, "-w", 1, "-r", 2, "--pp-schedule", "1f1b", "--dp-buckets", "2")
    assert d["global"]["pp_schedule"] == "1f1b" and len(d["ranks"]) == w


@pytest.mark.parametrize("sched", ["gpipe", "1f1b"])
def test_moe_ep_overlap(sched, data_dir):
    base = run(4, "hybrid_3d_moe", "tiny_moe_8_bfloat16", 2, 4, 2, data_dir, "-w", 1, "-r", 2, "--pp-schedule", sched)
    d = run(4, "hybrid_3d_moe", "tiny_moe_8_bfloat16", 2, 4, 2, data_dir, "-w", 1, "-r", 2, "--pp-schedule", sched,
            "--ep-overlap")
    assert d["global"]["ep_overlap"] is True and base["global"]["ep_overlap"] is False
    for r0, r1 in zip(base["ranks"], d["ranks"]):
        assert len(r1["ep_comm_time"]) == 2 * len(r0["ep_comm_time"])  # two halves per chunk
        assert r1["comm"]["ep_alltoall"]["bytes_per_op"] * 2 == r0["comm"]["ep_alltoall"]["bytes_per_op"]


def test_1f1b_rejects_reference_schedule(data_dir):
    import subprocess
    p = subprocess.run([os.path.join(BIN, "hybrid_2d"), "tiny_dense_8_bfloat16", "1", "2", data_dir, "--pp-schedule",
                        "1f1b", "--schedule", "reference"], capture_output=True, text=True)
    assert p.returncode == 2 and "1f1b" in p.stderr


@pytest.mark.parametrize("w,S,T,gran", [(2, 1, 2, "microbatch"), (4, 2, 2, "microbatch"), (4, 2, 2, "layer"),
                                        (8, 2, 2, "microbatch")])
def test_hybrid_3d(w, S, T, gran, data_dir):
    mb = 2
    d = run(w, "hybrid_3d", "tiny_dense_8_bfloat16", S, mb, T, data_dir, "-w", 1, "-r", 2,
            "--tp-granularity", gran)
    g = d["global"]
    assert PP_GLOBAL | {"num_tensor_shards", "tp_allreduce_size_bytes"} <= set(g)
    assert g["tp_allreduce_size_bytes"] == 64 * 128 * (8 // mb) // T * 2
    assert g["dp_allreduce_size_bytes"] == (1000003 // (S * T)) * 2
    n_ar = 4 * mb if gran == "microbatch" else 2 * (4 // S) * 2 * mb
    for r in d["ranks"]:
        assert {"tp_comm_time", "tp_id", "dp_id"} <= set(r)
        assert len(r["tp_comm_time"]) == 2 * n_ar
        assert r["tp_id"] == r["rank"] % T


@pytest.mark.parametrize("w,S,EP", [(2, 1, 2), (4, 2, 2), (8, 2, 4)])
def test_hybrid_3d_moe(w, S, EP, data_dir):
    mb = 2
    d = run(w, "hybrid_3d_moe", "tiny_moe_8_bfloat16", S, mb, EP, data_dir, "-w", 1, "-r", 2)
    g = d["global"]
    assert PP_GLOBAL | {"num_expert_shards", "num_experts", "sequence_length", "embedded_dim",
                        "ep_alltoall_size_bytes"} <= set(g)
    assert g["num_experts"] == 4
    assert g["ep_alltoall_size_bytes"] == (8 // mb) * 64 * 2 * 128 // EP * 2
    ne = 400000 // S
    assert g["dp_allreduce_size_bytes"] == (ne + (2000000 - 400000) // S // EP) * 2
    for r in d["ranks"]:
        assert {"ep_comm_time", "dp_ep_comm_time", "ep_id", "dp_id"} <= set(r)
        assert len(r["ep_comm_time"]) == 2 * (2 * (4 // S) * mb * 2)
        assert len(r["dp_ep_comm_time"]) == 2


def test_hybrid_3d_moe_rejects_bad_expert_split(data_dir):
    code, outs = launch.launch(3, [os.path.join(BIN, "hybrid_3d_moe"), "tiny_moe_8_bfloat16", "1", "2", "3",
                                   data_dir, "--quiet"], timeout=60, capture=True)
    assert code != 0
    assert "divisible" in "".join(o or "" for o in outs)


def test_dp_options_inplace_optimizer_minexec(data_dir):
    d = run(2, "dp", "tiny_dense_8_bfloat16", 4, data_dir, "-w", 3, "-m", 0.05, "--in-place", "--optimizer")
    g = d["global"]
    assert g["in_place"] is True
    runs = g["dlnb"]["runs"]
    import math
    warm = g["dlnb"]["warmup_times"]
    assert runs >= math.ceil(0.05 / max(warm) - 1e-9)
    assert len(d["ranks"][0]["runtimes"]) == runs


def test_pipeline_dp_buckets(data_dir):
    d = run(4, "hybrid_2d", "tiny_dense_8_bfloat16", 2, 4, data_dir, "-w", 1, "-r", 2, "--dp-buckets", 4)
    for r in d["ranks"]:
        assert len(r["dp_comm_time"]) == 2 * 4


def test_loop_mode_terminates_with_max_iters(data_dir):
    code, outs = launch.launch(2, [os.path.join(BIN, "dp_loop"), "tiny_dense_8_bfloat16", "2", data_dir,
                                   "--quiet", "--max-loop-iters", "5"], timeout=60, capture=True)
    assert code == 0
    assert "DLNB_REPORT_BEGIN" not in outs[0]


def test_json_output_file(tmp_path, data_dir):
    out = tmp_path / "r.json"
    run(2, "dp", "tiny_dense_8_bfloat16", 2, data_dir, "-w", 0, "-r", 1, "--json", out)
    import json
    d = json.loads(out.read_text())
    assert d["section"] == "dp" and len(d["ranks"]) == 2


def test_gpt2_l_dp_cpu_baseline_config1(root):
    """BASELINE.json config 1: gpt2_l DP on the CPU backend, W = 2 (full-size buffers)."""
    d = run(2, "dp", "gpt2_l_16_bfloat16", 10, root, "-w", 1, "-r", 2, timeout=300)
    it = d["global"]["dlnb"]["iteration"]
    assert it["median_ms"] >= it["compute_floor_ms"] * 0.98
    assert d["global"]["msg_size_avg_bytes"] == 77403008 * 2


CP_GLOBAL = {"model_name", "num_cp_shards", "cp_algo", "local_batch_size", "world_size", "dp_size", "sequence_length",
             "local_sequence_length", "num_layers", "attention_fraction", "fwd_rt_per_layer", "bwd_rt_per_layer",
             "total_model_size_params", "num_dp_buckets", "dp_allreduce_size_bytes", "device", "backend"}
CP_RANK = {"runtimes", "cp_comm_time", "cp_exposed_time", "dp_comm_time", "dp_exposed_time", "cp_id", "dp_id", "hostname"}


@pytest.mark.parametrize("w,C,algo", [(2, 2, "ring"), (4, 2, "ring"), (4, 4, "ring"), (2, 2, "ulysses"),
                                      (4, 4, "ulysses"), (2, 1, "ring"), (8, 4, "ring"), (8, 4, "ulysses")])
def test_hybrid_cp(w, C, algo, data_dir):
    """Context parallelism (extension): ring attention P2P or Ulysses all-to-all + DP gradient buckets."""
    d = run(w, "hybrid_cp", "tiny_dense_8_bfloat16", C, data_dir, "-w", 1, "-r", 2, "--cp-algo", algo)
    g = d["global"]
    assert d["section"] == "dp_cp" and CP_GLOBAL <= set(g)
    assert g["num_cp_shards"] == C and g["dp_size"] == w // C and g["cp_algo"] == algo
    s_loc = 64 // C
    assert g["local_sequence_length"] == s_loc and g["num_layers"] == 4 and g["num_dp_buckets"] == 4
    if algo == "ring":
        assert g["cp_kv_block_size_bytes"] == 2 * 8 * s_loc * 128 * 2  # K+V, B=8, d_kv=d (no GQA), bf16
    else:
        assert g["cp_alltoall_qkv_size_bytes"] == 8 * s_loc * 3 * 128 * 2
        assert g["cp_alltoall_out_size_bytes"] == 8 * s_loc * 128 * 2
    floor_ms = 6.0 / C
    assert g["dlnb"]["iteration"]["compute_floor_ms"] == pytest.approx(floor_ms)
    assert sorted(r["cp_id"] for r in d["ranks"]) == sorted(r % C for r in range(w))
    for r in d["ranks"]:
        assert CP_RANK <= set(r)
        assert len(r["runtimes"]) == 2 and len(r["dp_exposed_time"]) == 2 and len(r["dp_comm_time"]) == 2
        assert len(r["cp_comm_time"]) == (2 if C > 1 else 0) and len(r["cp_exposed_time"]) == (2 if C > 1 else 0)
        for rt in r["runtimes"]:
            assert rt * 1e3 >= floor_ms * 0.98
        if C > 1:
            kinds = set(r["comm"])
            assert ("cp_ring_sendrecv" in kinds) if algo == "ring" else ("cp_alltoall_qkv" in kinds)
            # ring: 2 * L * (C - 1) sends per iteration; ulysses: 4 * L all-to-alls
            first = "cp_ring_sendrecv" if algo == "ring" else "cp_alltoall_qkv"
            assert r["comm"][first]["ops"] == 2 * (4 * (C - 1) if algo == "ring" else 2 * 4)


def test_hybrid_cp_rejects_bad_split(data_dir):
    code, outs = launch.launch(3, [os.path.join(BIN, "hybrid_cp"), "tiny_dense_8_bfloat16", "3", data_dir, "--quiet"],
                               timeout=60, capture=True)
    assert code != 0 and "seq_len 64 must be divisible by num_cp_shards 3" in "".join(o or "" for o in outs)


@pytest.mark.parametrize("w,S,mb,T,E,extra", [(8, 2, 2, 2, 2, []), (4, 1, 2, 2, 2, []),
                                              (4, 2, 4, 2, 1, ["--pp-schedule", "1f1b"]),
                                              (4, 1, 2, 2, 2, ["--tp-granularity", "layer"]),
                                              (8, 1, 2, 2, 2, [])])
def test_hybrid_4d(w, S, mb, T, E, extra, data_dir):
    """DP x PP x TP x EP (extension): TP fastest, then EP, then stage, then DP."""
    d = run(w, "hybrid_4d", "tiny_moe_8_bfloat16", S, mb, T, E, data_dir, "-w", 1, "-r", 2, *extra)
    g = d["global"]
    assert d["section"] == "dp_pp_tp_ep" and PP_GLOBAL <= set(g)
    assert g["num_tensor_shards"] == T and g["num_expert_shards"] == E and g["dp_size"] == w // (S * T * E)
    spmb = 8 // mb
    pipe = 64 * 128 * spmb
    assert g["pipe_msg_size_bytes"] == pipe * 2 and g["tp_allreduce_size_bytes"] == pipe // T * 2
    assert g["ep_alltoall_size_bytes"] == spmb * 64 * 2 * 128 // E // T * 2
    ne = 400000 // S // T
    assert g["ep_allreduce_size_bytes"] == ne * 2
    assert g["dp_allreduce_size_bytes"] == (ne + (1600000 // S) // E // T) * 2
    assert g["dlnb"]["iteration"]["compute_floor_ms"] == pytest.approx((mb + S - 1) * 6.0 / S / (mb * T))
    coords = sorted((r["tp_id"], r["ep_id"], r["stage_id"], r["dp_id"]) for r in d["ranks"])
    expect = sorted((r % T, (r // T) % E, (r // (T * E)) % S, r // (T * E * S)) for r in range(w))
    assert coords == expect
    layer = "layer" in extra
    # TP all-reduces per microbatch and direction: 2 (reference granularity) or 2 per layer; x 2 directions x 2 runs
    n_tp = (2 * (4 // S) if layer else 2) * mb * 2 * 2
    for r in d["ranks"]:
        assert len(r["runtimes"]) == 2
        assert len(r["tp_comm_time"]) == n_tp
        assert len(r["ep_comm_time"]) == 2 * (4 // S) * mb * 2 * 2


@pytest.mark.parametrize("prog,model,params", [("hybrid_3d", "tiny_dense_8_bfloat16", (2, 2, 2)),
                                               ("hybrid_4d", "tiny_moe_8_bfloat16", (1, 2, 2, 2))])
def test_sequence_parallel(prog, model, params, data_dir):
    """--sequence-parallel (Megatron-SP): every TP all-reduce becomes all-gather + reduce-scatter of 1/T shards."""
    base = run(4, prog, model, *params, data_dir, "-w", 1, "-r", 2)
    d = run(4, prog, model, *params, data_dir, "-w", 1, "-r", 2, "--sequence-parallel")
    assert d["global"]["sequence_parallel"] is True and base["global"]["sequence_parallel"] is False
    T = params[2]
    tp = d["global"]["tp_allreduce_size_bytes"] // 2
    for r, rb in zip(d["ranks"], base["ranks"]):
        c = r["comm"]
        assert "tp_allreduce" not in c and c["tp_allgather"]["ops"] == c["tp_reduce_scatter"]["ops"]
        assert c["tp_allgather"]["ops"] == rb["comm"]["tp_allreduce"]["ops"]
        assert c["tp_allgather"]["bytes_per_op"] == -(-tp // T) * T * 2
        assert len(r["tp_comm_time"]) == len(rb["tp_comm_time"])


@pytest.mark.parametrize("w,S,mb,V", [(2, 2, 2, 2), (4, 2, 4, 2), (2, 2, 4, 3), (4, 4, 4, 3), (4, 4, 8, 2),
                                      (8, 4, 4, 2), (1, 1, 2, 4)])
def test_interleaved_1f1b(w, S, mb, V, data_dir):
    """--pp-schedule interleaved (extension): V model chunks per stage, wrap link, bubble / V."""
    d = run(w, "hybrid_2d", "tiny_deep_8_bfloat16", S, mb, data_dir, "-w", 1, "-r", 2, "--pp-schedule", "interleaved",
            "--pp-virtual", V)
    g = d["global"]
    assert g["pp_schedule"] == "interleaved" and g["pp_virtual_stages"] == V
    f_mb, b_mb = 2.0 / S / mb, 4.0 / S / mb  # ms (tiny tables: fwd 2 ms, bwd 4 ms)
    floor = (mb + (S - 1) / V) * (f_mb + b_mb)
    assert g["dlnb"]["iteration"]["compute_floor_ms"] == pytest.approx(floor)
    for r in d["ranks"]:
        assert len(r["pp_comm_time"]) == 2 * 2 * mb * V  # one per chunk forward / backward, 2 runs
        for rt in r["runtimes"]:
            assert rt * 1e3 >= floor * 0.98


def _fails(n, prog, *args):
    code, outs = launch.launch(n, [os.path.join(BIN, prog), *map(str, args), "--quiet"], timeout=60, capture=True)
    return code, "".join(o or "" for o in outs)


def test_extension_argument_checks(data_dir):
    code, out = _fails(4, "hybrid_2d", "tiny_deep_8_bfloat16", 4, 2, data_dir, "--pp-schedule", "interleaved")
    assert code != 0 and "num_microbatches 2 must be a multiple of num_stages 4" in out
    code, out = _fails(2, "hybrid_2d", "tiny_dense_8_bfloat16", 2, 2, data_dir, "--pp-schedule", "interleaved",
                       "--pp-virtual", 4)
    assert code != 0 and "must be divisible by stages*virtual 8" in out
    code, out = _fails(4, "hybrid_4d", "tiny_moe_8_bfloat16", 1, 2, 2, 2, data_dir, "--ep-overlap")
    assert code != 0 and "--ep-overlap is not supported with tensor parallelism" in out
    code, out = _fails(4, "hybrid_4d", "tiny_moe_8_bfloat16", 1, 2, 2, 3, data_dir)
    assert code != 0
    code, out = _fails(2, "hybrid_cp", "tiny_dense_8_bfloat16", 2, data_dir, "--cp-algo", "bogus")
    assert code != 0 and "--cp-algo must be ring or ulysses" in out


def test_extensions_other_wire_dtypes_and_reference_schedule(data_dir):
    d = run(2, "dp", "tiny_dense_8_bfloat16", 3, data_dir, "-w", 0, "-r", 1, "--zero", 2, "--wire-dtype", "fp32")
    assert d["global"]["param_allgather_msg_size_bytes"] == -(-333335 // 2) * 2 * 4
    d = run(2, "hybrid_cp", "tiny_dense_8_bfloat16", 2, data_dir, "-w", 0, "-r", 1, "--schedule", "reference")
    assert d["global"]["dlnb"]["schedule"] == "reference"
    d = run(4, "hybrid_4d", "tiny_moe_8_bfloat16", 2, 2, 2, 1, data_dir, "-w", 0, "-r", 1, "--pp-schedule", "interleaved",
            "--pp-virtual", 2)
    assert d["global"]["pp_virtual_stages"] == 2


@pytest.mark.parametrize("w,params,alpha", [(4, (1, 2, 4), 1.0), (8, (2, 2, 4), 2.0)])
def test_moe_expert_imbalance(w, params, alpha, data_dir):
    """--ep-imbalance: Zipf-skewed dispatch as an all-to-allv (grouped send/recv)."""
    d = run(w, "hybrid_3d_moe", "tiny_moe_8_bfloat16", *params, data_dir, "-w", 1, "-r", 2, "--ep-imbalance", alpha)
    g = d["global"]
    E = params[2]
    per = g["ep_dispatch_bytes_per_peer"]
    assert g["ep_imbalance"] == alpha and len(per) == E
    assert all(a > b for a, b in zip(per, per[1:]))  # EP rank 0 hosts the hot experts
    assert sum(per) == g["ep_alltoall_size_bytes"] * E  # same tokens as the uniform all-to-all
    assert per[0] / per[-1] == pytest.approx(E ** alpha, rel=0.01)
    for r in d["ranks"]:
        assert r["ep_comm_time"] and all(t >= 0 for t in r["ep_comm_time"])


def test_moe_expert_imbalance_argument_checks(data_dir):
    p = subprocess.run([os.path.join(BIN, "hybrid_3d_moe"), "tiny_moe_8_bfloat16", "1", "2", "1", data_dir,
                        "--ep-imbalance", "-1"], capture_output=True, text=True)
    assert p.returncode == 1 and "ep-imbalance" in p.stderr


@pytest.mark.parametrize("w,prog,model,params", [(2, "hybrid_2d", "tiny_deep_8_bfloat16", (2, 4)),
                                                 (4, "hybrid_2d", "tiny_deep_8_bfloat16", (4, 8)),
                                                 (8, "hybrid_2d", "tiny_deep_8_bfloat16", (4, 8)),
                                                 (8, "hybrid_3d", "tiny_dense_8_bfloat16", (2, 4, 2)),
                                                 (8, "hybrid_3d_moe", "tiny_moe_8_bfloat16", (2, 4, 2))])
def test_dualpipe(w, prog, model, params, data_dir):
    """--pp-schedule dualpipe: bidirectional pipeline, mirrored stage pairs sum their gradients."""
    d = run(w, prog, model, *params, data_dir, "-w", 1, "-r", 2, "--pp-schedule", "dualpipe")
    g = d["global"]
    assert g["pp_schedule"] == "dualpipe" and g["dualpipe_ticks"] >= params[1]
    it = g["dlnb"]["iteration"]
    S, mb = params[0], params[1]
    f, b = g["fwd_rt_per_microbatch"], g["bwd_rt_per_microbatch"]
    # the schedule's compute floor: at least mb (f + b), and below 1F1B's (mb + S - 1)(f + b) for S >= 4
    assert it["compute_floor_ms"] * 1e3 >= mb * (f + b) - 1e-6
    if S >= 4:
        assert it["compute_floor_ms"] * 1e3 < (mb + S - 1) * (f + b)
    moe = prog == "hybrid_3d_moe"
    for r in d["ranks"]:
        assert len(r["runtimes"]) == 2
        if moe:
            # EP all-reduce of the non-expert gradients first, then the whole pair / DP sync
            assert r["dualpipe_early_sync_tick"] == -1
            assert len(r["pp_mirror_time"]) == 2 and len(r["dp_comm_time"]) == 2
        else:
            # two mirror all-reduces and two DP all-reduces per iteration: the
            # early half is issued mid-backward (before this stage's last
            # backward tick), the rest after the backward
            assert len(r["pp_mirror_time"]) == 2 * 2 and len(r["dp_comm_time"]) == 2 * 2
            assert 0 <= r["dualpipe_early_sync_tick"] < r["dualpipe_last_backward_tick"]


@pytest.mark.parametrize("params,extra,msg", [((3, 6), [], "even number of stages"),
                                              ((2, 3), [], "even number of microbatches"),
                                              ((2, 4), ["--dp-buckets", "2"], "dp-buckets")])
def test_dualpipe_argument_checks(params, extra, msg, data_dir):
    code, outs = launch.launch(params[0], [os.path.join(BIN, "hybrid_2d"), "tiny_deep_8_bfloat16",
                                           *map(str, params), data_dir, "--pp-schedule", "dualpipe", *extra,
                                           "--quiet"], timeout=60, capture=True)
    text = "".join(o or "" for o in outs)
    assert code != 0 and msg in text, text[-2000:]


def test_dualpipe_native_floor_matches_model(data_dir):
    """The native driver's tick count and compute floor equal the Python model's for the same f, b."""
    from dlnetbench_amd.parallel import schedule_sim as sim
    S, mb = 4, 8
    d = run(S, "hybrid_2d", "tiny_deep_8_bfloat16", S, mb, data_dir, "-w", 1, "-r", 1, "--pp-schedule", "dualpipe")
    g = d["global"]
    f, b = g["fwd_rt_per_microbatch"], g["bwd_rt_per_microbatch"]
    assert g["dualpipe_ticks"] == len(sim.dualpipe_ticks(S, mb))
    assert g["dlnb"]["iteration"]["compute_floor_ms"] * 1e3 == pytest.approx(sim.dualpipe_floor(S, mb, f, b), rel=1e-6)


@pytest.mark.parametrize("w,prog,model,params", [(4, "hybrid_2d", "tiny_deep_8_bfloat16", (4, 8)),
                                                 (8, "hybrid_3d_moe", "tiny_moe_8_bfloat16", (2, 4, 2))])
def test_dualpipe_planner_matches_native(w, prog, model, params, data_dir):
    """plan.py --pp-schedule dualpipe: doubled DP gradient, pair all-reduce and compute floor as the native run."""
    import json as _json
    from dlnetbench_amd.parallel import plan as P
    from dlnetbench_amd.utils.stats import load_stats
    d = run(w, prog, model, *params, data_dir, "-w", 1, "-r", 1, "--pp-schedule", "dualpipe")
    st = load_stats(os.path.join(data_dir, "model_stats", model + ".txt"))
    with open(os.path.join(data_dir, "models", model.rsplit("_", 2)[0] + ".json")) as f:
        arch = _json.load(f)
    L = arch.get("num_encoder_blocks", 0) + arch.get("num_decoder_blocks", 0)
    inner = params[2] if len(params) > 2 else 1
    pl = P.plan_hybrid(st, w, prog, params[0], params[1], inner, L, pp_schedule="dualpipe")
    msgs = {m.name: m for m in pl.messages}
    comm = d["ranks"][0]["comm"]
    assert comm["dp_allreduce"]["bytes_per_op"] == msgs["dp_allreduce"].wire_bytes
    assert comm["pp_mirror_allreduce"]["bytes_per_op"] == msgs["pp_mirror_allreduce"].wire_bytes
    assert comm["pp_mirror_allreduce"]["nranks"] == 2
    floor_ms = d["global"]["dlnb"]["iteration"]["compute_floor_ms"]
    assert pl.compute_per_unit_us["compute_floor_us"] / 1e3 == pytest.approx(floor_ms, rel=1e-6)


def test_dp_geometric_buckets_split_flops_like_time(data_dir):
    """--dp-bucket-ratio < 1: every bucket's backward FLOPs (what --compute flops executes) take the same share
    as its time and its parameters (the FLOPs stayed backward_flops / nb)."""
    d = run(1, "dp", "tiny_dense_8_bfloat16", 4, data_dir, "--backend", "cpu", "--dp-bucket-ratio", "0.5",
            "--compute", "flops", "-w", "0", "-r", "1")
    g = d["global"]
    sizes, us, fl = g["bucket_sizes"], g["bwd_us_per_bucket"], g["bwd_flops_per_bucket"]
    P = g["total_model_size_params"]
    assert len(sizes) == len(us) == len(fl) == 4 and sizes[0] > sizes[-1]
    for sz, u, f in zip(sizes, us, fl):
        assert u / us[0] == pytest.approx(sz / sizes[0], rel=1e-9)
        assert f / fl[0] == pytest.approx(sz / sizes[0], rel=1e-9)
    assert sum(us) == pytest.approx(4 * g["bwd_rt_per_bucket"], rel=1e-9)
    assert sum(sizes) == P


def test_stream_task_failure_raises_in_process_and_next_run_works(data_dir):
    """A failing CPU-stream task in a library host (engine.run in this interpreter) raises NativeError
    instead of ending the process; the next job in the same process runs normally."""
    import time
    from dlnetbench_amd import engine
    from dlnetbench_amd._native import NativeError
    kw = dict(base_path=data_dir, backend="cpu", compute="sleep", warmup=1, runs=3, silent=True)
    # the same job before the fault, in this process and under the same host load: the yardstick for "normal"
    before = engine.run("fsdp", "tiny_dense_8_bfloat16", 4, 1, **kw)["global"]["dlnb"]["iteration"]
    os.environ["DLNB_INJECT_FAULT"] = "rank=0,iter=1,mode=task"
    try:
        with pytest.raises(NativeError, match="injected fault in a stream task"):
            engine.run("fsdp", "tiny_dense_8_bfloat16", 4, 1, **kw)
    finally:
        del os.environ["DLNB_INJECT_FAULT"]
    t0 = time.time()
    d = engine.run("fsdp", "tiny_dense_8_bfloat16", 4, 1, **kw)
    it = d["global"]["dlnb"]["iteration"]
    assert it["compute_floor_ms"] <= it["timed_ms_per_iter"]
    # no leftover of the failed job slows it: within 2x + 20 ms of the clean run (a loaded CI host, e.g. pytest -n)
    assert it["timed_ms_per_iter"] < 2 * before["timed_ms_per_iter"] + 20
    assert time.time() - t0 < 20


def test_comm_delay_fault_raises_exposed_timers(data_dir, monkeypatch):
    """DLNB_COMM_FAULT mode=delay (an idle task of X after the operation on its stream): a delay on the
    operation an exposed-communication timer waits for raises that timer by X - here DP's last all-reduce of
    every iteration (barrier_time) and FSDP's last reduce-scatter (barrier) on 2 CPU ranks, X = 100 ms. Several
    specs (';') hit different ops; every=N picks the K-th op of every iteration. (CPU worker threads of 2
    ranks x 3 streams on a shared, possibly loaded host: only the lower bounds are load-proof - the delayed
    operation lasts >= X and the wait for it >= X; tests/test_gpu_timers.py checks the device timers to
    0.03 ms.)"""
    X = 100.0
    monkeypatch.setenv("DLNB_COMM_FAULT", "mode=delay,us=100000,op=all_reduce,call=4,every=5")
    slow = run(2, "dp", "tiny_dense_8_bfloat16", 5, data_dir, "-w", 1, "-r", 4)
    for r in slow["ranks"]:
        ar = [x * 1e3 for x in r["allreduce_time"]]
        assert all(ar[k] >= X for k in range(4, len(ar), 5)), ar
        assert min(r["barrier_time"]) * 1e3 >= 0.9 * X, r["barrier_time"]
    monkeypatch.setenv("DLNB_COMM_FAULT", "mode=delay,us=100000,op=reduce_scatter,call=3,every=4;"
                                          "mode=delay,us=1000,op=all_gather,call=99999")
    slow_f = run(2, "fsdp", "tiny_dense_8_bfloat16", 4, 2, data_dir, "-w", 1, "-r", 4)
    for r in slow_f["ranks"]:
        assert min(r["barrier"]) * 1e3 >= 0.9 * X, r["barrier"]


def test_comm_delay_fault_argument_checks(data_dir, monkeypatch):
    for spec, msg in [("mode=delay,op=all_reduce", "us=X"), ("mode=delay,us=5,op=bogus", "unknown op"),
                      ("mode=swap,op=send", "op=send only")]:
        monkeypatch.setenv("DLNB_COMM_FAULT", spec)
        code, outs = launch.launch(1, [os.path.join(BIN, "dp"), "tiny_dense_8_bfloat16", "5", data_dir, "-w", "1",
                                       "-r", "1", "--quiet"], timeout=60, capture=True)
        assert code != 0
