"""8192^3 bf16 GEMM launches for PMC runs: variant (waves selector) from argv[1], 10 launches each."""
import sys
import torch
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm

M = N = K = 8192
a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
gemm.fill_random_(a, 1)
gemm.fill_random_(b, 2)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
for v in [int(x) for x in sys.argv[1].split(",")]:
    for _ in range(10):
        gemm.gemm_tn(a, b, c, waves=v)
torch.cuda.synchronize()
print("done", flush=True)
