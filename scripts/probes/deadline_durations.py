"""Event-timed duration of gemm_deadline_us / idle_wait_us for several targets, 5 repeats each."""
import sys
import torch
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm

a = torch.empty(8192, 4096, device="cuda", dtype=torch.bfloat16)
b = torch.empty(14336, 4096, device="cuda", dtype=torch.bfloat16)
gemm.fill_random_(a, 1)
gemm.fill_random_(b, 2)
c = torch.empty(8192, 14336, device="cuda", dtype=torch.bfloat16)
st = torch.zeros(8, dtype=torch.int64, device="cuda")
s = torch.cuda.current_stream()
for name, fn in (("idle", lambda us: gemm.idle_wait_us(us)), ("gemm", lambda us: gemm.gemm_deadline_us(a, b, c, us, st))):
    for us in (100.0, 200.0, 2000.0):
        out = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            fn(us)
            e1.record(s)
            torch.cuda.synchronize()
            out.append(round(e0.elapsed_time(e1) * 1e3, 1))
        print(name, us, out, flush=True)
