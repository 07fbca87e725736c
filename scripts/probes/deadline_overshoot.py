"""Where a deadline GEMM's extra time goes: device-clock stamps around gemm_deadline_us.

For each launch: s0 = stamp before, t0 = first block's start (the epoch slot's low 48 bits),
s1 = stamp after. start latency = t0 - s0, overshoot = s1 - (t0 + ticks). 100 MHz ticks -> us.
DLNB_GEMM_8PHASE=0|1 selects the kernel."""
import sys
import torch
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm

a = torch.empty(8192, 4096, device="cuda", dtype=torch.bfloat16)
b = torch.empty(14336, 4096, device="cuda", dtype=torch.bfloat16)
gemm.fill_random_(a, 1)
gemm.fill_random_(b, 2)
c = torch.empty(8192, 14336, device="cuda", dtype=torch.bfloat16)
slot = torch.zeros(8, dtype=torch.int64, device="cuda")
st = torch.zeros(8, dtype=torch.int64, device="cuda")
for us in (100.0, 500.0, 2000.0):
    lat, over = [], []
    for rep in range(8):
        gemm.stamp_(st, 0)
        gemm.gemm_deadline_us(a, b, c, us, slot)
        gemm.stamp_(st, 1)
        torch.cuda.synchronize()
        s0, s1 = st[0].item(), st[1].item()
        t0 = slot[0].item() & ((1 << 48) - 1)
        s0 &= (1 << 48) - 1
        s1 &= (1 << 48) - 1
        lat.append((t0 - s0) / 100.0)
        over.append((s1 - t0) / 100.0 - us)
    print(f"us={us}: start latency {sorted(lat)[4]:.2f} us (min {min(lat):.2f}), "
          f"overshoot median {sorted(over)[4]:.2f} us (min {min(over):.2f}, max {max(over):.2f})", flush=True)
