"""Throughput of the hand-written MFMA GEMM vs torch (hipBLASLt) on MI355X.

    python -m dlnetbench_amd.tools.gemm_bench [--shapes 8192x14336x4096,...] [--dtype bf16|fp8]

Interleaves the two implementations round by round in one process
(cdna_hip_programming.md §5.4 rule 24) on random [-1, 1) operands (rule 25)
and prints TFLOP/s (median, best) as JSON lines. Variants: ours = 8 waves double
buffered (default), ours_alt = the variant under test (bf16: software-pipelined
fragment reads, waves=2; fp8: the 3-deep A ring, waves=1), ours4 = 4 waves.
"""
from __future__ import annotations

import argparse
import json
import statistics


def main(argv=None) -> int:
    import torch
    from dlnetbench_amd.ops import gemm

    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="4096x4096x4096,8192x8192x8192,8192x14336x4096,8192x28672x8192,2048x5120x1280")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"])
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=20)
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

        def ours():
            gemm.gemm_tn(A, B, C, waves=8)

        def ours8():
            gemm.gemm_tn(A, B, C, waves=2 if dt == torch.bfloat16 else 1)

        def ours4():
            gemm.gemm_tn(A, B, C, waves=4)

        if dt == torch.bfloat16:
            def ref():
                torch.matmul(A, B.t(), out=C)
        else:
            one = torch.ones((), device="cuda", dtype=torch.float32)

            def ref():
                torch._scaled_mm(A, B.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)

        res = {"ours": [], "ours_alt": [], "ours4": [], "torch": []}
        for fn in (ours, ours8, ours4, ref):  # warm
            for _ in range(3):
                fn()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for name, fn in (("ours", ours), ("ours_alt", ours8), ("ours4", ours4), ("torch", ref)):
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
