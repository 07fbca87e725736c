"""Python reader for model_stats/*.txt (all three layouts, by key).

Mirrors the native parser (csrc/src/workload.cpp): the reference reads the
file positionally (cpp/utils.hpp:200-269) and its generator writes another
layout (python/model_stats.py:153-166); keys make both unambiguous.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict


@dataclass
class ModelStats:
    path: str
    format: str
    forward_flops: float
    backward_flops: float
    model_size: int
    non_expert_size: int
    fwd_us: float
    bwd_us: float
    batch: int
    ffn_fwd_us: float
    ffn_bwd_us: float
    experts: int
    seq_len: int
    hidden: int
    device: str = ""
    dtype: str = ""
    bytes_per_element: float = 2.0
    num_layers: int = 0
    ffn_dim: int = 0


_ORDER = ["forward_flops", "backward_flops", "model_size", "non_expert_size", "average_forward_time",
          "average_backward_time", "batch_size", "ffn_average_forward_time", "ffn_average_backward_time",
          "experts", "seq_len", "embedded_dim"]


def _canon(k: str) -> str:
    out = []
    for c in k:
        if c in " (":
            break
        out.append(c.lower())
    return "".join(out)


def parse_stats_text(text: str, origin: str = "<text>") -> ModelStats:
    kv: Dict[str, str] = {}
    idx = 0
    for raw in text.splitlines():
        line = raw.strip()
        if not line or line.startswith("#"):
            continue
        if ":" not in line:
            raise ValueError(f"{origin}: line without ':' : {line!r}")
        k, v = line.split(":", 1)
        key = _canon(k.strip()) or (_ORDER[idx] if idx < len(_ORDER) else f"line{idx}")
        kv[key] = v.strip()
        idx += 1

    def need(k):
        if k not in kv:
            raise ValueError(f"{origin}: missing key {k}")
        return kv[k]

    experts = int(float(kv.get("experts", "1"))) or 1
    model_size = int(need("model_size"))
    if "non_expert_size" in kv:
        ne = int(kv["non_expert_size"])
        fmt = "dlnb" if "generator" in kv else "shipped"
    else:
        fmt = "generator"
        ne = model_size if experts > 1 else 0
    st = ModelStats(
        path=origin, format=fmt,
        forward_flops=float(need("forward_flops")), backward_flops=float(need("backward_flops")),
        model_size=model_size, non_expert_size=ne,
        fwd_us=float(need("average_forward_time")), bwd_us=float(need("average_backward_time")),
        batch=int(need("batch_size")),
        ffn_fwd_us=float(kv.get("ffn_average_forward_time", 0)), ffn_bwd_us=float(kv.get("ffn_average_backward_time", 0)),
        experts=experts, seq_len=int(need("seq_len")), hidden=int(need("embedded_dim")),
        device=kv.get("device", ""), dtype=kv.get("dtype", ""),
        bytes_per_element=float(kv.get("bytes_per_element", 2.0)),
        num_layers=int(kv.get("num_layers", 0)), ffn_dim=int(kv.get("ffn_dim", 0)),
    )
    if st.batch <= 0:
        raise ValueError(f"{origin}: Batch_size must be > 0")
    return st


def load_stats(path: str) -> ModelStats:
    with open(path) as f:
        return parse_stats_text(f.read(), path)
