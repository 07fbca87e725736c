"""Tile-order group size of the 8-phase GEMM (DLNB_GEMM_GROUP: M-tiles that
share B panels in L2), interleaved rounds in one process, random operands.
usage: gemm_group.py bf16|fp8 [groups, default 4,8,16,32]"""
import os
import statistics
import sys
import torch
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm

dt = sys.argv[1]
groups = [int(g) for g in (sys.argv[2] if len(sys.argv) > 2 else "4,8,16,32").split(",")]
for M, N, K in ((4096, 4096, 4096), (8192, 8192, 8192), (8192, 14336, 4096)):
    A = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
    B = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
    gemm.fill_random_(A, 1)
    gemm.fill_random_(B, 2)
    if dt == "fp8":
        A, B = A.to(torch.float8_e4m3fn), B.to(torch.float8_e4m3fn)
    C = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
    res = {g: [] for g in groups}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rnd in range(7):
        for g in groups:
            os.environ["DLNB_GEMM_GROUP"] = str(g)
            gemm.gemm_tn(A, B, C)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(20):
                gemm.gemm_tn(A, B, C)
            e1.record()
            torch.cuda.synchronize()
            res[g].append(2.0 * M * N * K * 20 / (e0.elapsed_time(e1) * 1e-3) / 1e12)
    print({"M": M, "N": N, "K": K, "dtype": dt,
           **{f"g{g}": round(statistics.median(v), 1) for g, v in res.items()}}, flush=True)
