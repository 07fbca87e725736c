"""Deadline accuracy of the persistent GEMM stand-in per shape: event-timed duration of
gemm_deadline_us(500 us) (median of 20), for bf16 and fp8 at the llama3-8B FFN and ViT-H FFN
shapes. Prints one JSON line per case."""
import json
import statistics
import sys

import torch

sys.path.insert(0, ".")
from dlnetbench_amd.ops import gemm  # noqa: E402

US = 500.0
for dt in ("bf16", "fp8"):
    for (M, N, K) in ((8192, 14336, 4096), (8192, 5120, 1280), (8192, 1280, 5120)):
        a = torch.empty(M, K, device="cuda", dtype=torch.bfloat16)
        b = torch.empty(N, K, device="cuda", dtype=torch.bfloat16)
        gemm.fill_random_(a, 1)
        gemm.fill_random_(b, 2)
        if dt == "fp8":
            a, b = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
        c = torch.empty(M, N, device="cuda", dtype=torch.bfloat16)
        stamp = torch.zeros(8, dtype=torch.int64, device="cuda")
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for _ in range(3):
            gemm.gemm_deadline_us(a, b, c, US, stamp)
        t = []
        for _ in range(20):
            e0.record(s)
            gemm.gemm_deadline_us(a, b, c, US, stamp)
            e1.record(s)
            torch.cuda.synchronize()
            t.append(e0.elapsed_time(e1) * 1e3)
        print(json.dumps({"dtype": dt, "shape": f"{M}x{N}x{K}", "target_us": US, "median_us": round(statistics.median(t), 1),
                          "max_us": round(max(t), 1)}), flush=True)
