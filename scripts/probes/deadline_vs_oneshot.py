"""Workload for a PMC comparison of the bf16 deadline GEMM (the headline's
compute) with the one-shot kernel of the same shape.

    python3 scripts/probes/deadline_vs_oneshot.py oneshot|deadline [M N K [bf16|fp8]]

oneshot: 10 back-to-back gemm_tn launches (variant 0, all CUs);
deadline: 5 x 20-ms persistent deadline launches on CUs - 32 (the bench's grid).
Run under rocprofv3 --pmc (scripts/probes/deadline_pmc.sh) and merge with
tools/prof_merge.py."""
import sys

import torch

sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm  # noqa: E402

mode = sys.argv[1]
M, N, K = (int(x) for x in sys.argv[2:5]) if len(sys.argv) > 4 else (8192, 14336, 4096)
fp8 = len(sys.argv) > 5 and sys.argv[5] == "fp8"
a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
gemm.fill_random_(a, 1)
gemm.fill_random_(b, 2)
if fp8:
    a, b = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
if mode == "oneshot":
    for _ in range(10):
        gemm.gemm_tn(a, b, c)
else:
    stamp = torch.zeros(8, dtype=torch.int64, device="cuda")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for _ in range(5):
        gemm.gemm_deadline_us(a, b, c, 20000.0, stamp, grid=cus - 32)
torch.cuda.synchronize()
