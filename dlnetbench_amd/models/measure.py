"""Measured workload generator: stats tables timed on the local GPU.

    python -m dlnetbench_amd.models.measure llama3_8b --batch_size 16 [--dtype bfloat16|float8] [--out DIR]
    python -m dlnetbench_amd.models.measure --all-models --out model_stats_measured

The reference derives compute durations from a B200 roofline only
(python/model_stats.py:47-61,137-140; SURVEY.md §7.1 "optional measured
mode"). This times the real thing on an MI355X instead: ONE decoder/encoder
block of the architecture (random init, torch on ROCm: hipBLASLt GEMMs,
flash SDPA) at the full batch and sequence length, forward and
forward+backward, scaled by the layer count, plus the embedding / LM-head
(or patch-embedding / pooler) cost timed separately. Mixtral's MoE layer
routes tokens with a real top-2 router and runs every expert on its tokens.
float8 times the block's linear layers with ``torch._scaled_mm`` (OCP e4m3,
per-tensor scales) and keeps attention in bf16.

The file has the same layout as the roofline generator (FLOP counts stay the
reference's analytic ones so compute-by-FLOPs modes agree), with
``Generator:dlnetbench_amd.models.measure device=<name>``.
"""
from __future__ import annotations

import argparse
import math
import os
import statistics
from typing import Callable, List, Tuple

from .registry import MODELS, ModelArch, get_model
from .roofline import BYTES, Stats, compute_stats


def _timer(torch, fn: Callable[[], None], reps: int, warmup: int = 2) -> float:
    """Median seconds per call of fn (CUDA events around each call)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e-3)
    return statistics.median(ts)


def _linear(torch, fp8: bool):
    """y = x @ w.T, in bf16 or through fp8 _scaled_mm (autograd-capable)."""
    F = torch.nn.functional

    class Fp8Linear(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x, w):
            ctx.save_for_backward(x, w)
            one = torch.ones((), device=x.device, dtype=torch.float32)
            x8 = x.reshape(-1, x.shape[-1]).to(torch.float8_e4m3fn)
            w8 = w.to(torch.float8_e4m3fn)
            y = torch._scaled_mm(x8, w8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            return y.reshape(*x.shape[:-1], w.shape[0])

        @staticmethod
        def backward(ctx, gy):
            x, w = ctx.saved_tensors
            one = torch.ones((), device=x.device, dtype=torch.float32)
            g2 = gy.reshape(-1, gy.shape[-1])
            x2 = x.reshape(-1, x.shape[-1])
            g8 = g2.to(torch.float8_e4m3fn)
            # dX = dY @ W  (W^T given as column-major operand), dW = dY^T @ X
            wt8 = w.t().contiguous().to(torch.float8_e4m3fn)
            dx = torch._scaled_mm(g8, wt8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            gt8 = g2.t().contiguous().to(torch.float8_e4m3fn)
            xt8 = x2.t().contiguous().to(torch.float8_e4m3fn)
            dw = torch._scaled_mm(gt8, xt8.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            return dx.reshape(x.shape), dw

    if not fp8:
        return lambda x, w: F.linear(x, w)
    return Fp8Linear.apply


class _Block:
    """Parameters + forward of one block of `m` (random init, bf16)."""

    def __init__(self, torch, m: ModelArch, fp8: bool):
        self.t, self.m = torch, m
        dev, dt = "cuda", torch.bfloat16
        d, f, hd = m.hidden, m.ffn, m.head_dim
        kvd = m.kv * hd

        def P(*shape):
            return (torch.randn(*shape, device=dev, dtype=dt) * (1.0 / math.sqrt(shape[-1]))).requires_grad_(True)

        self.lin = _linear(torch, fp8)
        if m.family in ("gpt2", "vit"):
            self.wqkv, self.wo = P(3 * d, d), P(d, d)
            self.w1, self.w2 = P(f, d), P(d, f)
            self.params = [self.wqkv, self.wo, self.w1, self.w2]
        else:
            self.wq, self.wk, self.wv, self.wo = P(d, d), P(kvd, d), P(kvd, d), P(d, d)
            E = m.experts
            self.router = P(E, d) if E > 1 else None
            self.w_gate = [P(f, d) for _ in range(E)]
            self.w_up = [P(f, d) for _ in range(E)]
            self.w_down = [P(d, f) for _ in range(E)]
            self.params = [self.wq, self.wk, self.wv, self.wo] + self.w_gate + self.w_up + self.w_down
            if self.router is not None:
                self.params.append(self.router)

    def forward(self, x):
        t, m = self.t, self.m
        F = t.nn.functional
        B, N, d = x.shape
        H, hd = m.heads, m.head_dim
        causal = m.family != "vit"
        if m.family in ("gpt2", "vit"):
            h = F.layer_norm(x, (d,))
            q, k, v = self.lin(h, self.wqkv).split(d, dim=-1)
            kvh = H
        else:
            h = F.rms_norm(x, (d,))
            q, k, v = self.lin(h, self.wq), self.lin(h, self.wk), self.lin(h, self.wv)
            kvh = m.kv
        q = q.view(B, N, H, hd).transpose(1, 2)
        k = k.view(B, N, kvh, hd).transpose(1, 2)
        v = v.view(B, N, kvh, hd).transpose(1, 2)
        if kvh != H:
            k = k.repeat_interleave(H // kvh, dim=1)
            v = v.repeat_interleave(H // kvh, dim=1)
        a = F.scaled_dot_product_attention(q, k, v, is_causal=causal)
        x = x + self.lin(a.transpose(1, 2).reshape(B, N, d), self.wo)
        if m.family in ("gpt2", "vit"):
            h = F.layer_norm(x, (d,))
            return x + self.lin(F.gelu(self.lin(h, self.w1)), self.w2)
        h = F.rms_norm(x, (d,)).reshape(B * N, d)
        if m.experts == 1:
            y = self.lin(F.silu(self.lin(h, self.w_gate[0])) * self.lin(h, self.w_up[0]), self.w_down[0])
            return x + y.view(B, N, d)
        # top-k routing, every expert on its tokens (index_add combine)
        logits = F.linear(h, self.router)
        w, idx = t.topk(t.softmax(logits.float(), dim=-1), m.top_k, dim=-1)
        y = t.zeros_like(h)
        for e in range(m.experts):
            tok, slot = (idx == e).nonzero(as_tuple=True)
            if tok.numel() == 0:
                continue
            he = h[tok]
            ye = self.lin(F.silu(self.lin(he, self.w_gate[e])) * self.lin(he, self.w_up[e]), self.w_down[e])
            y = y.index_add(0, tok, ye * w[tok, slot].unsqueeze(-1).to(ye.dtype))
        return x + y.view(B, N, d)


def _edge_costs(torch, m: ModelArch, B: int) -> Tuple[float, float]:
    """(fwd, bwd) seconds of what is outside the blocks, in bf16: embedding
    gather + LM head + log-softmax (LMs, in token chunks with per-chunk
    backward so the logits never exist all at once) or patch embedding +
    pooler (ViT)."""
    dev, dt = "cuda", torch.bfloat16
    F = torch.nn.functional
    d, N = m.hidden, m.seq_len
    if m.family == "vit":
        px = torch.randn(B * (N - 1), 3 * m.patch_size ** 2, device=dev, dtype=dt)
        wp = (torch.randn(d, 3 * m.patch_size ** 2, device=dev, dtype=dt) * 0.02).requires_grad_(True)
        wpool = (torch.randn(d, d, device=dev, dtype=dt) * 0.02).requires_grad_(True)
        cls = torch.randn(B, d, device=dev, dtype=dt)

        def run(backward: bool):
            loss = F.linear(px, wp).float().sum() + torch.tanh(F.linear(cls, wpool)).float().sum()
            if backward:
                loss.backward()
                wp.grad = wpool.grad = None
    else:
        emb = (torch.randn(m.vocab, d, device=dev, dtype=dt) * 0.02).requires_grad_(True)
        head = emb if m.tie_embeddings else (torch.randn(m.vocab, d, device=dev, dtype=dt) * 0.02).requires_grad_(True)
        ids = torch.randint(0, m.vocab, (B * N,), device=dev)
        chunk = max(1, min(B * N, (1 << 31) // (m.vocab * 6)))  # ~2 GB of logits per chunk

        def run(backward: bool):
            h = emb[ids]
            hd = h.detach().requires_grad_(backward)
            for i in range(0, B * N, chunk):
                loss = F.linear(hd[i:i + chunk], head).float().logsumexp(-1).sum()
                if backward:
                    loss.backward()
            if backward:
                h.backward(hd.grad)
                emb.grad = None
                head.grad = None
    t_f = _timer(torch, lambda: run(False), reps=3)
    t_fb = _timer(torch, lambda: run(True), reps=3)
    return t_f, max(t_fb - t_f, 0.0)


def measure_stats(m: ModelArch, batch: int, dtype: str = "bfloat16", reps: int = 5) -> Stats:
    import torch
    assert torch.cuda.is_available(), "measured mode needs a GPU"
    fp8 = dtype == "float8"
    torch.manual_seed(0)
    blk = _Block(torch, m, fp8)
    x = torch.randn(batch, m.seq_len, m.hidden, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    t_f = _timer(torch, lambda: blk.forward(x), reps)

    def fb():
        blk.forward(x).float().sum().backward()
        for p in blk.params:
            p.grad = None
        x.grad = None
    t_fb = _timer(torch, fb, reps)
    e_f, e_b = _edge_costs(torch, m, batch)
    fwd = m.layers * t_f + e_f
    bwd = m.layers * max(t_fb - t_f, 0.0) + e_b
    roof = compute_stats(m, batch, dtype if dtype in ("bfloat16", "float8") else "bfloat16", "b200")
    props = torch.cuda.get_device_properties(0)
    arch = getattr(props, "gcnArchName", "").split(":")[0]
    # the marketing name is often just "AMD Radeon Graphics" (no amdgpu.ids on the box)
    name = "AMD Instinct MI355X (gfx950)" if arch == "gfx950" else f"{torch.cuda.get_device_name(0)} ({arch})"
    st = Stats(
        forward_flops=roof.forward_flops, backward_flops=roof.backward_flops, model_size=roof.model_size,
        non_expert_size=roof.non_expert_size, fwd_us=fwd * 1e6, bwd_us=bwd * 1e6, batch=batch,
        ffn_fwd_us=roof.ffn_fwd_us * (fwd / (roof.fwd_us * 1e-6)) if roof.fwd_us else 0.0,
        ffn_bwd_us=roof.ffn_bwd_us * (bwd / (roof.bwd_us * 1e-6)) if roof.bwd_us else 0.0,
        experts=m.experts, seq_len=m.seq_len, hidden=m.hidden, device=f"{name} (measured)", dtype=dtype,
        bytes_per_element=BYTES[dtype], layers=m.layers, ffn=m.ffn, top_k=m.top_k if m.experts > 1 else 1,
        preset="measured",
    )
    del blk, x
    torch.cuda.empty_cache()
    return st


def write_measured(out_dir: str, m: ModelArch, batch: int, dtype: str, reps: int = 5) -> str:
    os.makedirs(out_dir, exist_ok=True)
    st = measure_stats(m, batch, dtype, reps)
    lines = st.lines()
    lines[-1] = "Generator:dlnetbench_amd.models.measure device=" + st.device
    path = os.path.join(out_dir, f"{m.name}_{batch}_{dtype}.txt")
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")
    return path


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="Measured workload generator (stats timed on this GPU)")
    ap.add_argument("model", nargs="?", help="model name; omit with --all-models")
    ap.add_argument("--batch_size", "--batch-size", type=int, default=16)
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float8"])
    ap.add_argument("--all-models", action="store_true")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default="model_stats_measured")
    a = ap.parse_args(argv)
    models: List[ModelArch] = list(MODELS.values()) if a.all_models else [get_model(a.model)] if a.model else []
    if not models:
        ap.error("give a model or --all-models")
    for m in models:
        p = write_measured(a.out, m, a.batch_size, a.dtype, a.reps)
        print(p, flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
