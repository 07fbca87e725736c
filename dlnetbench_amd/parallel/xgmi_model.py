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
and return the predicted iteration time and exposed communication. They are
the numbers to hold the driver's measured scaling run against, and the way to
size DP buckets for point-to-point links instead of a switch
(`suggest_buckets`).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List

from ..utils.stats import ModelStats
from .plan import WIRE_BYTES, dp_bucket_sizes, fsdp_shards


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
