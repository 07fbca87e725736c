"""Throughput of the hand-written MFMA GEMM variants vs torch (hipBLASLt) on MI355X.

    python -m dlnetbench_amd.tools.gemm_bench [--shapes 8192x14336x4096,...] [--dtype bf16|fp8]
                                              [--variants 0,8]

Interleaves the implementations round by round in one process
(cdna_hip_programming.md §5.4 rule 24) on random [-1, 1) operands (rule 25)
and prints TFLOP/s (median, best) as JSON lines, one key per variant
(``v<n>_tflops_*``, n = the variant of ops.gemm.gemm_tn, csrc/include/dlnb/kernels.hpp:
0 = the default - with 256 x 32nf narrow tiles where square ones leave CUs
idle -, 5 = one wave per SIMD MX (fp8), 6 = 8-phase, 8 = 8 waves
double-buffered) and ``torch_tflops_*``.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics


def main(argv=None) -> int:
    import torch
    from dlnetbench_amd.ops import gemm

    ap = argparse.ArgumentParser()
    # square shapes, the headline stand-in (llama3-8B FFN down), and the skinny C5 stand-in (ViT-H FFN down,
    # narrow tiles)
    ap.add_argument("--shapes", default="4096x4096x4096,8192x8192x8192,8192x14336x4096,8192x4096x14336,"
                                        "8192x1280x5120,2048x5120x1280")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--variants", default=None, help="comma list of gemm_tn variants (default: 0,8 bf16; 0,6 fp8)")
    ap.add_argument("--ab", default=None, metavar="ENV=v1,v2",
                    help="run every variant once per value of a kernel environment knob read at launch "
                         "(e.g. DLNB_G4_OPT=0,3), interleaved; keys v<n>_<value>_tflops_*")
    a = ap.parse_args(argv)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float8_e4m3fn
    for shp in a.shapes.split(","):
        M, N, K = map(int, shp.split("x"))
        A = torch.empty(M, K, device="cuda", dtype=dt)
        B = torch.empty(N, K, device="cuda", dtype=dt)
        gemm.fill_random_(A, 1)
        gemm.fill_random_(B, 2)
        C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        flop = 2.0 * M * N * K

        variants = [int(v) for v in (a.variants or ("0,8" if a.dtype == "bf16" else "0,6")).split(",")]

        def mk(v, env=None):
            if env is None:
                return lambda: gemm.gemm_tn(A, B, C, waves=v)

            def fn():
                os.environ[env[0]] = env[1]  # putenv: the launch reads it
                gemm.gemm_tn(A, B, C, waves=v)
            return fn

        if a.ab:
            knob, vals = a.ab.split("=", 1)
            fns = [(f"v{v}_{x}", mk(v, (knob, x))) for v in variants for x in vals.split(",")]
        else:
            fns = [(f"v{v}", mk(v)) for v in variants]
        if dt == torch.bfloat16:
            def ref():
                torch.matmul(A, B.t(), out=C)
        else:
            one = torch.ones((), device="cuda", dtype=torch.float32)

            def ref():
                torch._scaled_mm(A, B.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
        fns.append(("torch", ref))
        res = {name: [] for name, _ in fns}
        for _, fn in fns:  # warm
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for name, fn in fns:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[name].append(flop * a.iters / (e0.elapsed_time(e1) * 1e-3) / 1e12)
        out = {"M": M, "N": N, "K": K, "dtype": a.dtype}
        for k, v in res.items():
            out[f"{k}_tflops_median"] = round(statistics.median(v), 1)
            out[f"{k}_tflops_best"] = round(max(v), 1)
        print(json.dumps(out), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
