"""Sustained MFMA rate of the persistent deadline GEMM (the bench's compute).

Runs gemm_deadline_us on the llama3-8B FFN-like shape for 5 x 20 ms.
Under `rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 ...` the MOPS counter
(x 512 FLOP) over the kernel time gives TFLOP/s. DLNB_GEMM_8PHASE=0|1
selects the schedule; argv[1] = fp8 runs the fp8 MX kernels."""
import sys
import torch
sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm

M, N, K = 8192, 14336, 4096
a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
gemm.fill_random_(a, 1)
gemm.fill_random_(b, 2)
if len(sys.argv) > 1 and sys.argv[1] == "fp8":
    a, b = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
stamp = torch.zeros(8, dtype=torch.int64, device="cuda")
for _ in range(5):
    gemm.gemm_deadline_us(a, b, c, 20000.0, stamp)
torch.cuda.synchronize()
print("done", flush=True)
