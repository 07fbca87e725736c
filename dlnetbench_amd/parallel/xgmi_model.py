"""Analytic cost model of the collectives on one 8 x MI355X node (xGMI mesh).

Every MI355X in a node has a direct xGMI link to each of the other 7 GPUs
(point-to-point, no switch). A collective over a group of n GPUs can therefore
spread its traffic over the n - 1 links that join the group's members:

* reduce-scatter / all-gather / all-to-all: each member exchanges 1/n of the
  per-op bytes with every other member, so each link carries S / n and
  t = S / n / (B * eta) + alpha;
* all-reduce = reduce-scatter + all-gather: t = 2 S / n / (B * eta) + 2 alpha;
* a ring (the algorithm a switch fabric favours) sends (n - 1) / n of S
  through ONE link per direction: t = (n - 1) / n * S / (B * eta) per phase;
* send / recv: one link, t = S / (B * eta) + alpha.

B is the per-link bandwidth per direction, eta the fraction of it a
collective achieves, alpha the per-collective latency. The defaults (153 GB/s,
0.75, 15 us) are assumptions to be replaced by `dlnb commtest --bench`
numbers from an 8-GPU node (--link-gbps / --eta / --alpha-us).

With our own kernels (`buffers` = "staged" for the xgmi backend's window
path, "registered" for its zero-copy path) a collective also moves local HBM
bytes, which can bound it before the links do: the per-rank traffic of each
kernel's data path (scripts/xgmi_roofline.py, measured at 81-104 % of the
D2D copy rate on one MI355X: profiles/xgmi_roofline_r2.md) over `hbm_gbps`,
and t = max(link time, HBM time) + alpha. "rccl" (default) is links only.

`predict_dp` / `predict_fsdp` replay the strategies' overlap schedules
(csrc/src/strategy_dp.cpp, strategy_fsdp.cpp: one in-order comm lane, a
collective waits for the compute that produced its data) with these times
and return the predicted iteration time and exposed communication.
`predict_hybrid` runs the pipeline schedules (schedule_sim, the enqueue
order of strategy_pipeline.cpp) with every stage-to-stage send/recv taking
its link time and the TP all-reduces / EP all-to-alls that sit on the
compute stream added to each microbatch's compute. They are
the numbers to hold the driver's measured scaling run against, and the way to
size DP buckets for point-to-point links instead of a switch
(`suggest_buckets`).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List

from ..utils.stats import ModelStats
from .plan import WIRE_BYTES, Plan, dp_bucket_sizes, fsdp_shards


@dataclass
class LinkModel:
    link_gbps: float = 153.0  # per link, per direction
    eta: float = 0.75
    alpha_us: float = 15.0
    gpus_per_node: int = 8
    buffers: str = "rccl"      # rccl | staged | registered (the xgmi kernels' data paths)
    hbm_gbps: float = 5000.0   # local HBM rate the kernels' copies reach (D2D copies: ~6 TB/s)

    def local_bytes(self, op: str, nbytes: float, n: int) -> float:
        """Local HBM bytes one rank's xgmi kernel moves (0 for rccl)."""
        if self.buffers == "rccl" or n <= 1:
            return 0.0
        blk = nbytes / n  # per-rank block of the gathered / reduced buffer
        if self.buffers == "registered":
            return {"allgather": blk * (n + 1), "reduce_scatter": blk * (n + 1), "alltoall": blk * (4 * n - 2),
                    "allreduce": 2.0 * nbytes, "sendrecv": 2.0 * nbytes}[op]
        return {"allgather": blk * (3 * n - 1), "reduce_scatter": blk * (3 * n - 1), "alltoall": blk * (4 * n - 2),
                "allreduce": nbytes * (6 * n - 4) / n, "sendrecv": 2.0 * nbytes}[op]

    def _bw(self) -> float:  # bytes per microsecond on one link
        return self.link_gbps * 1e3 * self.eta

    def coll_us(self, op: str, nbytes: float, n: int, algo: str = "direct") -> float:
        """Time of one collective whose algbw numerator is `nbytes` (the
        gathered / reduced buffer: count * n * elem for all-gather,
        reduce-scatter and all-to-all, count * elem for all-reduce)."""
        if n <= 1 or nbytes <= 0:
            return 0.0
        if n > self.gpus_per_node:
            raise ValueError("the model covers one node (at most %d GPUs per group)" % self.gpus_per_node)
        bw = self._bw()
        if op not in ("sendrecv", "allreduce", "allgather", "reduce_scatter", "alltoall"):
            raise ValueError(f"unknown op {op!r}")
        hbm = self.local_bytes(op, nbytes, n) / (self.hbm_gbps * 1e3)  # us
        if op == "sendrecv":
            return max(nbytes / bw, hbm) + self.alpha_us
        per_link = nbytes / n if algo == "direct" else nbytes * (n - 1) / n
        steps = 1 if algo == "direct" else (n - 1)
        if op == "allreduce":
            return max(2 * per_link / bw, hbm) + 2 * steps * self.alpha_us
        return max(per_link / bw, hbm) + steps * self.alpha_us


def predict_dp(st: ModelStats, world: int, nb: int, model: LinkModel, wire: str = "bf16",
               algo: str = "direct", ratio: float = 1.0) -> Dict[str, float]:
    """dp: forward, then bucket i's backward followed by its all-reduce on the
    comm lane (strategy_dp.cpp enqueue order); the iteration ends when the
    last all-reduce is done. ratio < 1: geometric buckets (--dp-bucket-ratio),
    each bucket's backward its share of the parameters."""
    es = WIRE_BYTES[wire]
    sizes = dp_bucket_sizes(st.model_size, nb, ratio)
    t = st.fwd_us
    lane = 0.0
    for s in sizes:
        t += st.bwd_us / nb if ratio >= 1.0 else st.bwd_us * s / st.model_size
        lane = max(lane, t) + model.coll_us("allreduce", s * es, world, algo)
    end = max(t, lane)
    floor = st.fwd_us + st.bwd_us
    return {"iter_ms": end / 1e3, "floor_ms": floor / 1e3, "exposed_ms": (end - floor) / 1e3,
            "allreduce_bucket_us": model.coll_us("allreduce", sizes[0] * es, world, algo)}


def predict_fsdp(st: ModelStats, world: int, U: int, F: int, model: LinkModel, wire: str = "bf16",
                 algo: str = "direct") -> Dict[str, float]:
    """fsdp with every collective of a rank on one in-order lane (the default
    `--comm-lanes single`), replaying csrc/src/strategy_fsdp.cpp: double-buffered
    gathers (all-gather u+1 waits for forward u-1 to release its buffer), the
    last unit stays gathered into the backward, all-gather u-1 is queued before
    the reduce-scatter of unit u, replica all-reduces follow their
    reduce-scatter, and the iteration ends when the lane drains."""
    es = WIRE_BYTES[wire]
    sh = fsdp_shards(st, U, F)
    ag = model.coll_us("allgather", sh[0] * F * es, F, algo)
    rs = model.coll_us("reduce_scatter", sh[0] * F * es, F, algo)
    R = world // F
    ar = model.coll_us("allreduce", sh[0] * es, R, algo) if R > 1 else 0.0
    f, b = st.fwd_us / U, st.bwd_us / U
    # forward
    lane = ag
    ready = {0: lane}
    fwd_end = {}
    t = 0.0
    for u in range(U):
        if u + 1 < U:
            lane = max(lane, fwd_end[u - 1] if u >= 1 else 0.0) + ag
            ready[u + 1] = lane
        t = max(t, ready[u]) + f
        fwd_end[u] = t
    # backward
    bwd_end, rs_end, ready_b = {}, {}, {}
    for u in range(U - 1, -1, -1):
        if u >= 1:
            lane = max(lane, bwd_end[u + 1] if u + 1 <= U - 1 else fwd_end[u - 1]) + ag
            ready_b[u - 1] = lane
        start = t if u == U - 1 else max(t, ready_b[u])
        if u + 2 <= U - 1:
            start = max(start, rs_end[u + 2])  # full_grad buffer reuse
        t = start + b
        bwd_end[u] = t
        lane = max(lane, t) + rs
        rs_end[u] = lane
        lane += ar
    end = max(t, lane)
    floor = st.fwd_us + st.bwd_us
    return {"iter_ms": end / 1e3, "floor_ms": floor / 1e3, "exposed_ms": (end - floor) / 1e3,
            "allgather_us": ag, "reduce_scatter_us": rs, "replica_allreduce_us": ar}


def suggest_buckets(st: ModelStats, world: int, model: LinkModel, wire: str = "bf16",
                    candidates: List[int] = (1, 2, 4, 8, 10, 16, 32, 64, 128)) -> Dict[str, float]:
    """DP bucket count with the lowest predicted iteration time: more buckets
    hide more of the all-reduce under the backward, each costs 2 alpha."""
    best = None
    for nb in candidates:
        p = predict_dp(st, world, nb, model, wire)
        if best is None or p["iter_ms"] < best[1]["iter_ms"] - 1e-9:
            best = (nb, p)
    return {"num_buckets": best[0], **best[1]}


def _ep_overlap_op_us(compute_us: float, n: int, half_us: float) -> float:
    """One microbatch's compute op under --ep-overlap (strategy_pipeline.cpp
    micro_compute): n slices of two halves; half hh's all-to-all runs on the EP
    lane after its compute slice, and its next slice waits for it; the op ends
    when both halves' last all-to-alls are done."""
    t_c = t_e = 0.0
    done = [0.0, 0.0]
    for i in range(n):
        for hh in (0, 1):
            t_c = (t_c if i == 0 else max(t_c, done[hh])) + compute_us / (2 * n)
            t_e = max(t_e, t_c) + half_us
            done[hh] = t_e
    return max(t_c, done[0], done[1])


def predict_hybrid(p: Plan, model: LinkModel, algo: str = "direct", pp_virtual: int = 1,
                   ep_overlap: bool = False) -> Dict[str, float]:
    """hybrid_2d / 3d / 3d_moe / 4d from their plan (plan.plan_hybrid): the
    schedule's makespan with the inner-group collectives on the compute stream
    (csrc/src/strategy_pipeline.cpp micro_compute: a microbatch's TP
    all-reduces and EP all-to-alls follow its compute in order, so they
    lengthen it) and every pipeline send/recv taking one link's time
    (rendezvous: both stages' link streams finish it together). The gradient
    all-reduces that end the iteration (DP, EP non-expert, DualPipe mirror)
    are added after the last backward, fully exposed: an upper bound when
    they are bucketed into the backward. ep_overlap: --ep-overlap's two
    half-microbatches, each all-to-all under the other half's compute
    (_ep_overlap_op_us)."""
    from . import schedule_sim as sim
    S, mb = p.params["num_stages"], p.params["num_microbatches"]
    sched = p.params.get("pp_schedule", "gpipe")
    V = pp_virtual if sched == "interleaved" else 1
    f, b = p.compute_per_unit_us["fwd_per_microbatch"], p.compute_per_unit_us["bwd_per_microbatch"]
    msgs = {m.name: m for m in p.messages}
    n_ops = mb * V  # forward (= backward) compute ops per rank per iteration
    inner = 0.0     # inner-group collective time per compute op
    for name in ("tp_allreduce", "ep_alltoall"):
        m = msgs.get(name)
        if m is not None:
            inner += m.calls_per_iter / (2 * n_ops) * model.coll_us(m.op, m.wire_bytes, m.group_size, algo)
    pipe = msgs.get("pipe_sendrecv")
    link = model.coll_us("sendrecv", pipe.wire_bytes, 2) if pipe is not None and S > 1 else 0.0
    fe, be = f + inner * V, b + inner * V  # build() splits f, b over the V chunks
    a2a = msgs.get("ep_alltoall")
    if ep_overlap:
        if a2a is None or "tp_allreduce" in msgs or sched == "dualpipe":
            raise ValueError("--ep-overlap applies to hybrid_3d_moe with gpipe / 1f1b / interleaved")
        n = a2a.calls_per_iter // (2 * n_ops)
        half = model.coll_us("alltoall", a2a.wire_bytes / 2, a2a.group_size, algo)
        fe = _ep_overlap_op_us(f / V, n, half) * V
        be = _ep_overlap_op_us(b / V, n, half) * V
        inner = (fe - f) / V
    if sched == "dualpipe":
        streams = sim.build_dualpipe(S, mb, fe, be, link)
    else:
        streams = sim.build(S, mb, V, fe, be, sched, link)
    span, stuck = sim.simulate(streams)
    if stuck:
        raise RuntimeError(f"{sched} schedule deadlocks in the model: {stuck[:4]}")
    tail = 0.0
    for name in ("pp_mirror_allreduce", "ep_nonexpert_allreduce", "dp_allreduce"):
        m = msgs.get(name)
        if m is not None and m.group_size > 1:
            tail += m.calls_per_iter * model.coll_us(m.op, m.wire_bytes, m.group_size, algo)
    floor = p.compute_per_unit_us["compute_floor_us"]
    end = span + tail
    return {"iter_ms": end / 1e3, "floor_ms": floor / 1e3, "exposed_ms": (end - floor) / 1e3,
            "inner_comm_per_op_us": inner, "sendrecv_us": link, "tail_allreduce_us": tail}


_FIT_OPS = {"all_reduce": "allreduce", "all_gather": "allgather", "reduce_scatter": "reduce_scatter",
            "all_to_all": "alltoall", "sendrecv": "sendrecv"}


def fit_link_model(lb: Dict[str, Dict[str, Dict[str, float]]], world: int, es: int = 2,
                   link_gbps: float = 153.0) -> Dict[str, object]:
    """eta and alpha of the direct-collective model from measured collective
    times: bench.py's link_bench for one backend ({op: {elements per rank:
    {"time_us", ...}}}, `dlnb commtest --bench` conventions). Every op's time
    is linear in its bytes under the model, t = steps * alpha + k * bytes /
    (B * eta) (k = 1/n for all-gather / reduce-scatter / all-to-all, 2/n for
    all-reduce, 1 for send/recv; steps 1 or 2), so two sizes give one
    (alpha, eta) per op; the medians over ops are the fit."""
    import statistics
    n = world
    per_op = {}
    for op, kind in _FIT_OPS.items():
        pts = []
        for count, v in (lb.get(op) or {}).items():
            if not isinstance(v, dict) or not v.get("time_us"):
                continue
            c = float(count)
            nbytes = c * es * (n if kind in ("allgather", "reduce_scatter", "alltoall") else 1)
            pts.append((nbytes, float(v["time_us"])))
        if len(pts) < 2 or n < 2:
            continue
        xs, ys = zip(*sorted(pts))
        mx, my = sum(xs) / len(xs), sum(ys) / len(ys)
        sxx = sum((x - mx) ** 2 for x in xs)
        if sxx <= 0:
            continue
        slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx  # us per byte
        icpt = my - slope * mx
        if slope <= 0:
            continue
        k = 1.0 if kind == "sendrecv" else (2.0 / n if kind == "allreduce" else 1.0 / n)
        steps = 2.0 if kind == "allreduce" else 1.0
        eta = k / (slope * link_gbps * 1e3)
        per_op[op] = {"eta": round(eta, 4), "alpha_us": round(max(0.0, icpt / steps), 2)}
    if not per_op:
        return {"eta": None, "alpha_us": None, "per_op": per_op}
    return {"eta": round(statistics.median(v["eta"] for v in per_op.values()), 4),
            "alpha_us": round(statistics.median(v["alpha_us"] for v in per_op.values()), 2),
            "per_op": per_op}

