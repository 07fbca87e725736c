"""Round 5: numerics of gemm_tn variant 9 (bf16 K-step planes) against fp32 torch, then throughput vs the 8-phase
default and hipBLASLt (gemm_bench)."""
import sys

import torch

from dlnetbench_amd.ops import gemm

bad = 0
for (M, N, K) in [(256, 256, 128), (256, 512, 128), (512, 512, 192), (768, 256, 256), (512, 256, 1024),
                  (768, 1280, 640), (2048, 1024, 4096), (256, 256, 192), (512, 768, 320)]:
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
    c = gemm.gemm_tn(a, b, waves=9)
    torch.cuda.synchronize()
    ref = a.float() @ b.float().t()
    err = (c.float() - ref).abs()
    bound = ref.abs() * 2 ** -8 + 1e-3 * ref.pow(2).mean().sqrt()
    ok = bool((err <= bound).all())
    bad += not ok
    print(f"{M}x{N}x{K}: {'ok' if ok else 'FAIL'} max err {err.max().item():.4g}", flush=True)
# identity: catches row / column swaps
a = torch.eye(256, 256, device="cuda", dtype=torch.bfloat16)
b = (torch.arange(256 * 256, device="cuda", dtype=torch.float32).reshape(256, 256) % 97 / 8.0).to(torch.bfloat16)
c = gemm.gemm_tn(a, b, waves=9)
torch.cuda.synchronize()
ident = torch.equal(c.float(), b.float().t())
print("identity", ident, flush=True)
sys.exit(1 if bad or not ident else 0)
