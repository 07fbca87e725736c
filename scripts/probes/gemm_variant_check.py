import torch, sys
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm
for dt in (torch.bfloat16, torch.float8_e4m3fn):
    for (M, N, K) in [(512, 768, 1024), (2048, 1024, 4096)]:
        a = (torch.randn(M, K, device="cuda") * 0.5).to(dt); b = (torch.randn(N, K, device="cuda") * 0.5).to(dt)
        ref = a.float() @ b.float().t()
        for v in (3, 6):
            c = gemm.gemm_tn(a, b, waves=v); torch.cuda.synchronize()
            err = (c.float() - ref).abs().max().item()
            print(dt, M, N, K, v, err, "OK" if err < 2e-2 * ref.abs().max().item() + 1e-2 else "BAD", flush=True)
