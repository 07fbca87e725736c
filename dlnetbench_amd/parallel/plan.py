"""Parallel layouts and message sizes, mirrored in Python.

These are the exact formulas the native drivers use (csrc/src/strategy_*.cpp),
which in turn follow the reference:

* DP   (cpp/data_parallel/dp.cpp:159-164): bucket i = P // nb (+1 for i < P % nb).
* FSDP (cpp/data_parallel/fsdp.cpp:244-265): unit u = P // U (+1 for u < P % U);
  shard = ceil(unit / F); unit group = rank // F; replica group = rank % F.
* Hybrids (hybrid_2d.cpp:236-282, hybrid_3d.cpp:283-325, hybrid_3d_moe.cpp:313-363):
  inner (TP/EP) fastest, then stage, then DP replica; pipe = s*d*B/mb;
  TP AR = pipe/T; DP AR = P/S, P/(S*T), NE/S + (P-NE)/S/EP; A2A per peer =
  (B/mb)*s*2*d/EP.

Used by the tests (golden values), by ``python -m dlnetbench_amd.parallel.plan``
(prints a run's messages, bytes and memory before launching it) and by the
results tooling (bus-bandwidth accounting).
"""
from __future__ import annotations

import argparse
import json
import math
import os
from dataclasses import asdict, dataclass, field
from typing import Dict, List

from ..utils.stats import ModelStats, load_stats

WIRE_BYTES = {"bf16": 2, "fp16": 2, "fp32": 4, "fp8": 1, "fp8_e4m3": 1, "fp8_e5m2": 1}


# --------------------------------------------------------------- layouts
def grid_coords(rank: int, inner: int, stages: int):
    """(inner_id, stage_id, dp_id) with inner fastest."""
    return rank % inner, (rank // inner) % stages, rank // (inner * stages)


def inner_group(rank: int, inner: int, stages: int) -> List[int]:
    i, s, d = grid_coords(rank, inner, stages)
    return [d * inner * stages + s * inner + k for k in range(inner)]


def pp_group(rank: int, inner: int, stages: int) -> List[int]:
    i, s, d = grid_coords(rank, inner, stages)
    return [d * inner * stages + k * inner + i for k in range(stages)]


def dp_group(rank: int, inner: int, stages: int, world: int) -> List[int]:
    i, s, d = grid_coords(rank, inner, stages)
    return [k * inner * stages + s * inner + i for k in range(world // (inner * stages))]


def fsdp_groups(rank: int, F: int, world: int):
    unit = [r for r in range(world) if r // F == rank // F]
    replica = [r for r in range(world) if r % F == rank % F]
    return unit, replica


# ----------------------------------------------------------------- plans
@dataclass
class Message:
    name: str
    op: str            # allreduce | allgather | reduce_scatter | alltoall | sendrecv
    group_size: int
    elements: int      # per-op element count in the reference's convention
    calls_per_iter: int
    wire_bytes: int = 0  # bytes moved by one op (algbw numerator)


@dataclass
class Plan:
    strategy: str
    world: int
    params: Dict[str, int]
    compute_per_unit_us: Dict[str, float]
    messages: List[Message] = field(default_factory=list)
    memory_bytes: int = 0

    def to_json(self) -> dict:
        d = asdict(self)
        return d


def _split(total: int, parts: int) -> List[int]:
    base, rem = divmod(total, parts)
    return [base + (1 if i < rem else 0) for i in range(parts)]


def dp_bucket_sizes(P: int, nb: int, ratio: float = 1.0) -> List[int]:
    """csrc/src/strategy_dp.cpp dp_bucket_sizes(), bit for bit: ratio 1 is the
    reference's P/nb partition (cpp/data_parallel/dp.cpp:159-164); ratio r < 1
    gives bucket i (backward order) floor(P r^i / sum_j r^j), the rest to
    bucket 0 (a geometric tail: the last, exposed all-reduce is small)."""
    if ratio >= 1.0:
        return _split(P, nb)
    w, x = [], 1.0
    for _ in range(nb):
        w.append(x)
        x *= ratio
    tot = 0.0
    for v in w:
        tot += v
    s = [int(math.floor(float(P) * v / tot)) for v in w]
    s[0] += P - sum(s)
    if min(s) <= 0:
        raise ValueError(f"--dp-bucket-ratio {ratio} leaves an empty bucket of {nb}")
    return s


def plan_dp(st: ModelStats, world: int, nb: int, wire: str = "bf16", zero: int = 0, ratio: float = 1.0) -> Plan:
    """zero = 1|2: ZeRO extension of csrc/src/strategy_dp.cpp (buckets padded to
    world * ceil(size / world); stage 2 reduce-scatters instead of all-reducing).
    ratio < 1: geometric bucket sizes (dp_bucket_sizes), listed per bucket."""
    es = WIRE_BYTES[wire]
    sizes = dp_bucket_sizes(st.model_size, nb, ratio)
    p = Plan("dp", world, {"num_buckets": nb, "zero": zero, "bucket_ratio": ratio},
             {"fwd": st.fwd_us, "bwd_per_bucket": st.bwd_us / nb})
    if ratio < 1.0:
        p.params["bucket_sizes"] = sizes
        p.compute_per_unit_us["bwd_per_bucket"] = [st.bwd_us * s / st.model_size for s in sizes]
    if not zero:
        p.messages.append(Message("bucket_allreduce", "allreduce", world, sizes[0], nb, sizes[0] * es))
        p.memory_bytes = 2 * st.model_size * es
        return p
    shard = -(-sizes[0] // world)
    if zero == 2:
        p.messages.append(Message("bucket_reduce_scatter", "reduce_scatter", world, shard, nb, shard * world * es))
    else:
        p.messages.append(Message("bucket_allreduce", "allreduce", world, shard * world, nb, shard * world * es))
    p.messages.append(Message("param_allgather", "allgather", world, shard, nb, shard * world * es))
    total = sum(-(-s // world) for s in sizes)
    # padded grads + (zero 1: reduced copy | zero 2: reduced shard) + param/momentum shards + gathered params
    p.memory_bytes = (2 * total * world + (total * world if zero == 1 else total) + 2 * total) * es
    return p


def fsdp_shards(st: ModelStats, U: int, F: int) -> List[int]:
    return [u // F + (1 if u % F else 0) for u in _split(st.model_size, U)]


def plan_fsdp(st: ModelStats, world: int, U: int, F: int, wire: str = "bf16") -> Plan:
    if world % F:
        raise ValueError("world size must be divisible by the sharding factor")
    es = WIRE_BYTES[wire]
    sh = fsdp_shards(st, U, F)
    R = world // F
    p = Plan("fsdp", world, {"num_units": U, "sharding_factor": F, "num_replicas": R},
             {"fwd_per_unit": st.fwd_us / U, "bwd_per_unit": st.bwd_us / U})
    p.messages.append(Message("allgather", "allgather", F, sh[0], 2 * U - 1, sh[0] * F * es))
    p.messages.append(Message("reduce_scatter", "reduce_scatter", F, sh[0], U, sh[0] * F * es))
    if R > 1:
        p.messages.append(Message("replica_allreduce", "allreduce", R, sh[0], U, sh[0] * es))
    p.memory_bytes = (2 * sum(sh) + 4 * sh[0] * F) * es
    return p


def ep_dispatch_counts(a2a: int, E: int, alpha: float) -> List[int]:
    """--ep-imbalance: elements every rank dispatches to EP rank j (Zipf 1/(j+1)^alpha
    of the uniform total a2a*E; the remainder goes to rank 0), as strategy_pipeline.cpp."""
    total = a2a * E
    if alpha <= 0 or E <= 1:
        return [a2a] * E
    w = [(1.0 + j) ** -alpha for j in range(E)]
    sw = sum(w)
    c = [int(total * x / sw) for x in w]
    c[0] += total - sum(c)
    return c


def plan_hybrid(st: ModelStats, world: int, kind: str, S: int, mb: int, inner: int = 1, layers: int = 0,
                wire: str = "bf16", tp_granularity: str = "microbatch", experts: int = 1,
                ep_imbalance: float = 0.0, pp_schedule: str = "gpipe", pp_virtual: int = 1) -> Plan:
    """hybrid_4d: inner = T (tensor shards), experts = E (expert shards); TP fastest, then EP.
    pp_schedule dualpipe (csrc/src/strategy_pipeline.cpp build_dualpipe): every rank holds two stage
    chunks, so its gradient (and non-expert part) doubles and mirrored stages s, S-1-s all-reduce it
    pairwise (in two halves) before the DP all-reduce. `compute_floor_us` is the schedule's makespan with free links.
    ep_imbalance > 0 (MoE): the all-to-all becomes an all-to-allv; the message's
    wire_bytes stay the uniform total and `ep_dispatch_elements_per_peer` gives the split."""
    if kind == "hybrid_4d":
        p = _plan_4d(st, world, S, mb, inner, experts, layers, wire, tp_granularity)
        return _apply_pp_schedule(p, S, mb, pp_schedule, pp_virtual, WIRE_BYTES[wire])
    es = WIRE_BYTES[wire]
    if layers and layers % S:
        raise ValueError("num_layers must be divisible by num_stages")
    if st.batch % mb:
        raise ValueError("batch must be divisible by num_microbatches")
    if world % (S * inner):
        raise ValueError("world must be divisible by stages*inner")
    spmb = st.batch // mb
    pipe = st.seq_len * st.hidden * spmb
    tsh = inner if kind == "hybrid_3d" else 1
    P = st.model_size
    params = {"num_stages": S, "num_microbatches": mb, "dp_size": world // (S * inner)}
    p = Plan(kind, world, params, {"fwd_per_microbatch": st.fwd_us / S / (mb * tsh),
                                   "bwd_per_microbatch": st.bwd_us / S / (mb * tsh)})
    if S > 1:
        p.messages.append(Message("pipe_sendrecv", "sendrecv", 2, pipe, 2 * mb, pipe * es))
    if kind == "hybrid_2d":
        dp_ar = P // S
    elif kind == "hybrid_3d":
        params["num_tensor_shards"] = inner
        dp_ar = P // (S * inner)
        tp = pipe // inner
        n = 4 * mb if tp_granularity == "microbatch" else 2 * (layers // S) * 2 * mb
        p.messages.append(Message("tp_allreduce", "allreduce", inner, tp, n, tp * es))
    else:
        params["num_expert_shards"] = inner
        ne = st.non_expert_size // S
        dp_ar = ne + ((P - st.non_expert_size) // S) // inner
        a2a = (spmb * st.seq_len * 2 * st.hidden) // inner
        p.messages.append(Message("ep_alltoall", "alltoall", inner, a2a, 2 * (layers // S) * mb * 2, a2a * inner * es))
        if ep_imbalance > 0:
            params["ep_dispatch_elements_per_peer"] = ep_dispatch_counts(a2a, inner, ep_imbalance)
        p.messages.append(Message("ep_nonexpert_allreduce", "allreduce", inner, ne, 1, ne * es))
    p.messages.append(Message("dp_allreduce", "allreduce", world // (S * inner), dp_ar, 1, dp_ar * es))
    p.memory_bytes = (8 * pipe + 2 * dp_ar) * es
    return _apply_pp_schedule(p, S, mb, pp_schedule, pp_virtual, es)


def _apply_pp_schedule(p: Plan, S: int, mb: int, sched: str, V: int, es: int) -> Plan:
    from . import schedule_sim as sim
    f, b = p.compute_per_unit_us["fwd_per_microbatch"], p.compute_per_unit_us["bwd_per_microbatch"]
    p.params["pp_schedule"] = sched
    if sched == "dualpipe":
        if S % 2 or mb % 2:
            raise ValueError("dualpipe needs an even number of stages and of microbatches")
        for m in p.messages:
            if m.name == "ep_nonexpert_allreduce":
                m.elements *= 2
                m.wire_bytes *= 2
        dp = next(m for m in p.messages if m.name == "dp_allreduce")
        p.memory_bytes += 2 * dp.elements * es  # the second chunk's gradient + buffer
        # the doubled gradient is synchronised in two halves (the early-finishing model stage mid-backward,
        # the other after the last backward), each a pair all-reduce followed by its DP all-reduce
        dp.calls_per_iter = 2
        p.messages.append(Message("pp_mirror_allreduce", "allreduce", 2, dp.elements, 2, dp.elements * es))
        p.compute_per_unit_us["compute_floor_us"] = sim.dualpipe_floor(S, mb, f, b)
    else:
        v = V if sched == "interleaved" else 1
        p.compute_per_unit_us["compute_floor_us"] = sim.floor(S, mb, v, f, b)
    return p


def _plan_4d(st: ModelStats, world: int, S: int, mb: int, T: int, E: int, layers: int, wire: str,
             tp_granularity: str) -> Plan:
    """DP x PP x TP x EP (csrc/src/strategy_pipeline.cpp, Hybrid4D)."""
    es = WIRE_BYTES[wire]
    if world % (S * T * E):
        raise ValueError("world must be divisible by stages*T*E")
    if st.batch % mb or (layers and layers % S):
        raise ValueError("batch % mb and layers % S must be 0")
    spmb = st.batch // mb
    pipe = st.seq_len * st.hidden * spmb
    lps = layers // S if layers else 1
    p = Plan("hybrid_4d", world, {"num_stages": S, "num_microbatches": mb, "num_tensor_shards": T,
                                  "num_expert_shards": E, "dp_size": world // (S * T * E)},
             {"fwd_per_microbatch": st.fwd_us / S / (mb * T), "bwd_per_microbatch": st.bwd_us / S / (mb * T)})
    if S > 1:
        p.messages.append(Message("pipe_sendrecv", "sendrecv", 2, pipe, 2 * mb, pipe * es))
    tp = pipe // T
    n_tp = (2 * lps if tp_granularity == "layer" else 2) * 2 * mb
    p.messages.append(Message("tp_allreduce", "allreduce", T, tp, n_tp, tp * es))
    a2a = (spmb * st.seq_len * 2 * st.hidden) // E // T
    p.messages.append(Message("ep_alltoall", "alltoall", E, a2a, 2 * lps * 2 * mb, a2a * E * es))
    ne = st.non_expert_size // S // T
    p.messages.append(Message("ep_nonexpert_allreduce", "allreduce", E, ne, 1, ne * es))
    dp_ar = ne + ((st.model_size - st.non_expert_size) // S) // E // T
    p.messages.append(Message("dp_allreduce", "allreduce", world // (S * T * E), dp_ar, 1, dp_ar * es))
    p.memory_bytes = (8 * pipe + 2 * dp_ar + 2 * a2a * E + 2 * tp) * es
    return p


def plan_cp(st: ModelStats, world: int, C: int, layers: int, heads: int, kv_heads: int, algo: str = "ring",
            buckets: int = 4, wire: str = "bf16") -> Plan:
    """DP x CP (csrc/src/strategy_cp.cpp): ring KV blocks or Ulysses all-to-alls per layer."""
    es = WIRE_BYTES[wire]
    if world % C or st.seq_len % C:
        raise ValueError("world and seq_len must be divisible by num_cp_shards")
    s_loc = st.seq_len // C
    dkv = st.hidden * kv_heads // heads
    p = Plan("hybrid_cp", world, {"num_cp_shards": C, "dp_size": world // C, "num_dp_buckets": min(buckets, layers)},
             {"fwd_per_layer": st.fwd_us / C / layers, "bwd_per_layer": st.bwd_us / C / layers})
    if C > 1:
        if algo == "ring":
            kv = 2 * st.batch * s_loc * dkv
            p.messages.append(Message("cp_ring_kv", "sendrecv", 2, kv, layers * (C - 1), kv * es))
            p.messages.append(Message("cp_ring_kv_dkv", "sendrecv", 2, 2 * kv, layers * (C - 1), 2 * kv * es))
        else:
            qkv = -(-st.batch * s_loc * (st.hidden + 2 * dkv) // C)
            out = -(-st.batch * s_loc * st.hidden // C)
            p.messages.append(Message("cp_alltoall_qkv", "alltoall", C, qkv, 2 * layers, qkv * C * es))
            p.messages.append(Message("cp_alltoall_out", "alltoall", C, out, 2 * layers, out * C * es))
    nb = min(buckets, layers)
    b0 = _split(st.model_size, nb)[0]
    p.messages.append(Message("dp_allreduce", "allreduce", world, b0, nb, b0 * es))
    p.memory_bytes = (st.model_size + 4 * st.batch * s_loc * max(dkv, st.hidden)) * es
    return p


def busbw_factor(op: str, n: int) -> float:
    """nccl-tests bus-bandwidth factor (BASELINE.md 'Metric definitions').

    0 for a single rank: nothing crosses a link (the op is a local copy)."""
    if n <= 1:
        return 0.0
    if op == "allreduce":
        return 2.0 * (n - 1) / n
    if op in ("allgather", "reduce_scatter", "alltoall"):
        return (n - 1) / n
    return 1.0


def model_layers(base: str, model: str) -> Dict[str, int]:
    """Layer and head counts of a stats-table model from its architecture JSON
    (models/<name>.json; the table name without its _<batch>_<dtype> suffix)."""
    name = model.rsplit("_", 2)[0]
    with open(os.path.join(base, "models", name + ".json")) as f:
        arch = json.load(f)
    heads = arch.get("num_heads", 1)
    return {"layers": arch.get("num_encoder_blocks", 0) + arch.get("num_decoder_blocks", 0), "heads": heads,
            "kv_heads": arch.get("dlnb", {}).get("num_kv_heads", heads)}


def predict(strategy: str, model: str, params: List[int], world: int, base: str = ".", wire: str = "bf16",
            algo: str = "direct", ep_overlap: bool = False, pp_schedule: str = "gpipe", pp_virtual: int = 2,
            dp_bucket_ratio: float = 1.0, **link) -> Dict[str, float]:
    """xGMI cost-model prediction (xgmi_model.py) of one run at `world` GPUs:
    dp, fsdp and the pipeline hybrids; `link` overrides LinkModel fields."""
    from . import xgmi_model as xm
    st = load_stats(os.path.join(base, "model_stats", model + ".txt"))
    lm = xm.LinkModel(**link)
    if strategy == "dp":
        return xm.predict_dp(st, world, params[0], lm, wire, algo, ratio=dp_bucket_ratio)
    if strategy == "fsdp":
        return xm.predict_fsdp(st, world, params[0], params[1], lm, wire, algo)
    if strategy in ("hybrid_2d", "hybrid_3d", "hybrid_3d_moe", "hybrid_4d"):
        L = model_layers(base, model)["layers"]
        inner = params[2] if len(params) > 2 else 1
        experts = params[3] if len(params) > 3 else 1
        pl = plan_hybrid(st, world, strategy, params[0], params[1], inner, L, wire=wire, experts=experts,
                         pp_schedule=pp_schedule, pp_virtual=pp_virtual)
        return xm.predict_hybrid(pl, lm, algo, pp_virtual, ep_overlap=ep_overlap)
    raise ValueError(f"no prediction for {strategy}")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Print the messages and memory of a benchmark run")
    ap.add_argument("strategy", choices=["dp", "fsdp", "hybrid_2d", "hybrid_3d", "hybrid_3d_moe", "hybrid_4d",
                                         "hybrid_cp"])
    ap.add_argument("model")
    ap.add_argument("params", nargs="+", type=int)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--base", default=".")
    ap.add_argument("--wire", default="bf16")
    ap.add_argument("--zero", type=int, default=0, help="dp: ZeRO stage 0|1|2")
    ap.add_argument("--dp-bucket-ratio", type=float, default=1.0,
                    help="dp: geometric bucket sizes, bucket i holds a share r^i (1 = the reference's P/nb)")
    ap.add_argument("--cp-algo", default="ring", choices=["ring", "ulysses"])
    ap.add_argument("--ep-imbalance", type=float, default=0.0, help="hybrid_3d_moe: Zipf exponent of the expert load")
    ap.add_argument("--pp-schedule", default="gpipe", choices=["gpipe", "1f1b", "interleaved", "dualpipe"])
    ap.add_argument("--pp-virtual", type=int, default=2, help="interleaved: model chunks per stage")
    ap.add_argument("--predict", action="store_true",
                    help="add the xGMI cost-model prediction (parallel/xgmi_model.py): dp / fsdp at W = 1, 2, 4, 8, "
                         "the pipeline hybrids at --world")
    ap.add_argument("--ep-overlap", action="store_true", help="hybrid_3d_moe --predict: dual-batch all-to-all overlap")
    ap.add_argument("--link-gbps", type=float, default=153.0, help="xGMI bandwidth per link and direction")
    ap.add_argument("--eta", type=float, default=0.75, help="achieved fraction of the link bandwidth")
    ap.add_argument("--alpha-us", type=float, default=15.0, help="latency per collective")
    ap.add_argument("--algo", default="direct", choices=["direct", "ring"])
    ap.add_argument("--buffers", default="rccl", choices=["rccl", "staged", "registered"],
                    help="--predict: add the local HBM traffic of the xgmi kernels' window (staged) or "
                         "zero-copy (registered) data path")
    ap.add_argument("--hbm-gbps", type=float, default=5000.0, help="--predict: local HBM rate of those kernels")
    a = ap.parse_args(argv)
    st = load_stats(os.path.join(a.base, "model_stats", a.model + ".txt"))
    if a.strategy == "dp":
        pl = plan_dp(st, a.world, *a.params, wire=a.wire, zero=a.zero, ratio=a.dp_bucket_ratio)
    elif a.strategy == "fsdp":
        pl = plan_fsdp(st, a.world, *a.params, wire=a.wire)
    else:
        ml = model_layers(a.base, a.model)
        L = ml["layers"]
        if a.strategy == "hybrid_cp":
            pl = plan_cp(st, a.world, a.params[0], L, ml["heads"], ml["kv_heads"], a.cp_algo, wire=a.wire)
        else:
            inner = a.params[2] if len(a.params) > 2 else 1
            experts = a.params[3] if len(a.params) > 3 else 1
            pl = plan_hybrid(st, a.world, a.strategy, a.params[0], a.params[1], inner, L, wire=a.wire,
                             experts=experts, ep_imbalance=a.ep_imbalance, pp_schedule=a.pp_schedule,
                             pp_virtual=a.pp_virtual)
    doc = pl.to_json()
    if a.predict and a.strategy in ("dp", "fsdp"):
        from . import xgmi_model as xm
        lm = xm.LinkModel(a.link_gbps, a.eta, a.alpha_us, buffers=a.buffers, hbm_gbps=a.hbm_gbps)
        pred = {}
        for w in (1, 2, 4, 8):
            if a.strategy == "dp":
                pred[str(w)] = xm.predict_dp(st, w, a.params[0], lm, a.wire, a.algo, ratio=a.dp_bucket_ratio)
            elif w % a.params[1] == 0 or a.params[1] == a.world:
                F = w if a.params[1] == a.world else a.params[1]  # fully sharded runs shard over the job
                pred[str(w)] = xm.predict_fsdp(st, w, a.params[0], F, lm, a.wire, a.algo)
        doc["xgmi_prediction"] = {"model": {"link_gbps": a.link_gbps, "eta": a.eta, "alpha_us": a.alpha_us,
                                            "algo": a.algo, "buffers": a.buffers, "hbm_gbps": a.hbm_gbps},
                                  "by_world": pred}
        if a.strategy == "dp":
            doc["xgmi_prediction"]["suggested_buckets_at_world"] = xm.suggest_buckets(st, a.world, lm, a.wire)
    elif a.predict and a.strategy.startswith("hybrid_") and a.strategy != "hybrid_cp":
        from . import xgmi_model as xm
        lm = xm.LinkModel(a.link_gbps, a.eta, a.alpha_us, buffers=a.buffers, hbm_gbps=a.hbm_gbps)
        doc["xgmi_prediction"] = {"model": {"link_gbps": a.link_gbps, "eta": a.eta, "alpha_us": a.alpha_us,
                                            "algo": a.algo, "buffers": a.buffers, "hbm_gbps": a.hbm_gbps},
                                  "at_world": a.world,
                                  "prediction": xm.predict_hybrid(pl, lm, a.algo, a.pp_virtual,
                                                                  ep_overlap=a.ep_overlap)}
    print(json.dumps(doc, indent=1))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
