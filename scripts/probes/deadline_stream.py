"""Sustained MFMA rate of the persistent deadline GEMM on one shape:
5 x 20 ms of gemm_deadline_us, grid = CUs - 32 (the bench's compute, which
leaves 32 CUs to collectives). Run under rocprofv3 --pmc with the MFMA MOPS
counters; DLNB_GEMM_STREAM=0|1 picks the per-tile or the streaming kernel.
usage: deadline_stream.py bf16|fp8 M N K"""
import sys
import torch
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm

dt, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
gemm.fill_random_(a, 1)
gemm.fill_random_(b, 2)
if dt == "fp8":
    a, b = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
stamp = torch.zeros(8, dtype=torch.int64, device="cuda")
grid = torch.cuda.get_device_properties(0).multi_processor_count - 32
for _ in range(5):
    gemm.gemm_deadline_us(a, b, c, 20000.0, stamp, grid=grid)
torch.cuda.synchronize()
print("done", flush=True)
