"""GEMM launches for PMC runs: our variants (waves selector) from argv[1], 10 launches each;
argv[2] = bf16 (default) | fp8; argv[3] = MxNxK (default 8192^3); variant "t" = torch (hipBLASLt:
matmul / _scaled_mm)."""
import sys
import torch
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm

M = N = K = 8192
if len(sys.argv) > 3:
    M, N, K = (int(x) for x in sys.argv[3].split("x"))
dt = sys.argv[2] if len(sys.argv) > 2 else "bf16"
a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
gemm.fill_random_(a, 1)
gemm.fill_random_(b, 2)
if dt == "fp8":
    a, b = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
one = torch.ones((), device="cuda", dtype=torch.float32)
for v in sys.argv[1].split(","):
    for _ in range(10):
        if v == "t":
            if dt == "fp8":
                torch._scaled_mm(a, b.t(), scale_a=one, scale_b=one, out_dtype=torch.bfloat16)
            else:
                torch.matmul(a, b.t())
        else:
            gemm.gemm_tn(a, b, c, waves=int(v))
torch.cuda.synchronize()
print("done", flush=True)
