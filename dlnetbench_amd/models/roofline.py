"""Roofline workload generator: writes model_stats/<model>_<B>_<dtype>.txt.

Same cost model as the reference (python/model_stats.py:47-61,116-140):
    attn_f = (8 B N d^2 + 4 B N^2 d) L        attn_b = (4 d^2 s + 2 B N d s) L
    mlp_f  = (4 B N d H k) L                  mlp_b  = (2 d H s E + 2 B N d s) L
    t = sum over {attn, mlp} of flops / min(peak, AI * BW);  t_bwd = 2 t_fwd
with k = 2 for Mixtral, E = experts, s = bytes per element.

Differences: the file is written in the layout the
runtime parses (15 shipped keys *including* Non_Expert_size), followed by
dlnb keys (Num_layers, FFN_dim, Top_k, Generator) that the reference's
positional parser would ignore. Parameter counts are analytic
(models/registry.py), so no weights are downloaded. Device presets:
``b200`` reproduces the reference's shipped tables; ``mi355x`` uses the
MI355X dense peaks (2.5 PF bf16, 5 PF fp8, 10 PF MX-fp4) and 8 TB/s.
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass
from typing import Dict, List

from .registry import MODELS, ModelArch, get_model


@dataclass(frozen=True)
class DevicePreset:
    name: str
    peaks: Dict[str, float]
    bandwidth: float


DEVICES: Dict[str, DevicePreset] = {
    # python/model_stats.py:19-26
    "b200": DevicePreset("NVIDIA B200-192GB (Single)",
                         {"bfloat16": 2.25e15, "float8": 4.5e15, "nvfp4": 9.0e15}, 8.0e12),
    # MI355X dense (non-sparse) peaks; MX-fp4 at 4x bf16 (MI355X_MICROARCH.md).
    "mi355x": DevicePreset("AMD Instinct MI355X (Single)",
                           {"bfloat16": 2.5e15, "float8": 5.0e15, "mxfp4": 10.0e15, "nvfp4": 10.0e15}, 8.0e12),
    # python/README.md:41-43 (the archived A100 tables)
    "a100": DevicePreset("NVIDIA A100-SXM4-80GB (Single)", {"bfloat16": 312e12}, 2.039e12),
}

BYTES = {"bfloat16": 2.0, "float8": 1.0, "nvfp4": 0.5, "mxfp4": 0.5}


def roofline_time(flops: float, bytes_accessed: float, peak: float, bw: float) -> float:
    ai = flops / bytes_accessed if bytes_accessed > 0 else float("inf")
    return flops / min(peak, ai * bw)


@dataclass
class Stats:
    forward_flops: int
    backward_flops: int
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
    device: str
    dtype: str
    bytes_per_element: float
    layers: int
    ffn: int
    top_k: int
    preset: str

    def lines(self) -> List[str]:
        return [
            f"Forward_Flops:{self.forward_flops}",
            f"Backward_Flops:{self.backward_flops}",
            f"Model_Size:{self.model_size}",
            f"Non_Expert_size:{self.non_expert_size}",
            f"Average_Forward_Time (us):{self.fwd_us:.2f}",
            f"Average_Backward_Time (us):{self.bwd_us:.2f}",
            f"Batch_size:{self.batch}",
            f"FFN_Average_Forward_Time (us):{self.ffn_fwd_us:.2f}",
            f"FFN_Average_Backward_Time (us):{self.ffn_bwd_us:.2f}",
            f"Experts:{self.experts}",
            f"Seq_len:{self.seq_len}",
            f"Embedded_dim:{self.hidden}",
            f"Device:{self.device}",
            f"Dtype:{self.dtype}",
            f"Bytes_per_element:{self.bytes_per_element}",
            f"Num_layers:{self.layers}",
            f"FFN_dim:{self.ffn}",
            f"Top_k:{self.top_k}",
            f"Generator:dlnetbench_amd.models.roofline preset={self.preset}",
        ]

    def text(self) -> str:
        return "\n".join(self.lines()) + "\n"


def compute_stats(model: ModelArch, batch: int, dtype: str = "bfloat16", preset: str = "b200") -> Stats:
    dev = DEVICES[preset]
    if dtype not in dev.peaks:
        raise ValueError(f"dtype {dtype!r} not supported by preset {preset!r}: {sorted(dev.peaks)}")
    B, N, d, H, L = batch, model.seq_len, model.hidden, model.ffn, model.layers
    E = model.experts
    k = model.top_k if model.experts > 1 else 1
    s = BYTES[dtype]
    peak = dev.peaks[dtype]
    attn_f = (8 * B * N * d ** 2 + 4 * B * N ** 2 * d) * L
    mlp_f = (4 * B * N * d * H * k) * L
    fwd_flops = attn_f + mlp_f
    attn_b = (4 * d ** 2 * s + 2 * B * N * d * s) * L
    mlp_b = (2 * d * H * s * E + 2 * B * N * d * s) * L
    t_attn = roofline_time(attn_f, attn_b, peak, dev.bandwidth)
    t_mlp = roofline_time(mlp_f, mlp_b, peak, dev.bandwidth)
    t_fwd = t_attn + t_mlp
    return Stats(
        forward_flops=int(fwd_flops), backward_flops=int(2 * fwd_flops),
        model_size=model.total_params(), non_expert_size=model.stats_non_expert(),
        fwd_us=t_fwd * 1e6, bwd_us=2 * t_fwd * 1e6, batch=B,
        ffn_fwd_us=t_mlp * 1e6, ffn_bwd_us=2 * t_mlp * 1e6,
        experts=E, seq_len=N, hidden=d, device=dev.name, dtype=dtype, bytes_per_element=s,
        layers=L, ffn=H, top_k=k, preset=preset,
    )


def write_stats(out_dir: str, model: ModelArch, batch: int, dtype: str, preset: str) -> str:
    os.makedirs(out_dir, exist_ok=True)
    st = compute_stats(model, batch, dtype, preset)
    path = os.path.join(out_dir, f"{model.name}_{batch}_{dtype}.txt")
    with open(path, "w") as f:
        f.write(st.text())
    return path


def write_arch_json(out_dir: str, model: ModelArch) -> str:
    import json
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, f"{model.name}.json")
    with open(path, "w") as f:
        json.dump(model.arch_json(), f, indent=2)
        f.write("\n")
    return path


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Roofline workload generator (model_stats/*.txt, models/*.json)")
    ap.add_argument("model", nargs="?", help="model name (e.g. llama3_8b or llama3-8b); omit with --all")
    ap.add_argument("--batch_size", "--batch-size", type=int, default=16)
    ap.add_argument("--dtype", default="bfloat16", choices=sorted(BYTES))
    ap.add_argument("--preset", default="b200", choices=sorted(DEVICES))
    ap.add_argument("--out", default="model_stats", help="output directory for stats files")
    ap.add_argument("--models-out", default=None, help="also write models/<name>.json here")
    ap.add_argument("--all", action="store_true", help="all models x batches {16,32,64,128} x {bfloat16,float8}")
    ap.add_argument("--list", action="store_true")
    a = ap.parse_args(argv)
    if a.list:
        for m in MODELS.values():
            print(f"{m.name:14s} {m.hf_name:40s} params={m.total_params():,}")
        return 0
    models = list(MODELS.values()) if a.all else [get_model(a.model)] if a.model else []
    if not models:
        ap.error("give a model or --all")
    batches = [16, 32, 64, 128] if a.all else [a.batch_size]
    dtypes = ["bfloat16", "float8"] if a.all else [a.dtype]
    for m in models:
        if a.models_out:
            write_arch_json(a.models_out, m)
        for b in batches:
            for dt in dtypes:
                p = write_stats(a.out, m, b, dt, a.preset)
                print(p)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
