"""Accuracy of the device-clock deadline kernels (idle wait, busy spin, MFMA GEMM).

    python -m dlnetbench_amd.tools.clock_check [--us 29320]
    python -m dlnetbench_amd.tools.clock_check --long-ms 2000 [--reps 5]

For each kernel: launch it back to back, time with HIP events and with the
host clock, print the relative error against the requested duration as JSON.
--long-ms: one idle wait of that length per rep, each bracketed by host
synchronizes, so a rate error of the deadline clock (kernels::wallclock_hz)
shows as ppm of host time (10 ppm = 20 us at 2 s; the launch + sync overhead,
~10-20 us, is the offset measured with a 1 ms wait).
"""
from __future__ import annotations

import argparse
import json
import statistics
import time


def _long(a) -> int:
    import torch
    from dlnetbench_amd import _native
    from dlnetbench_amd.ops import gemm

    def host_ms(us):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gemm.idle_wait_us(us)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3

    hz = _native.lib().dlnb_wallclock_hz(0)
    host_ms(1000.0)
    offset = statistics.median(host_ms(1000.0) - 1.0 for _ in range(5))  # launch + sync around a 1 ms wait
    errs = [host_ms(a.long_ms * 1e3) - offset - a.long_ms for _ in range(a.reps)]
    med = statistics.median(errs)
    print(json.dumps({"wallclock_hz": hz, "long_ms": a.long_ms, "offset_ms": round(offset, 4),
                      "err_us": [round(e * 1e3, 1) for e in errs], "err_us_median": round(med * 1e3, 1),
                      "err_ppm_median": round(med / a.long_ms * 1e6, 2)}), flush=True)
    return 0


def main(argv=None) -> int:
    import torch
    from dlnetbench_amd import _native
    from dlnetbench_amd.ops import gemm

    ap = argparse.ArgumentParser()
    ap.add_argument("--us", type=float, default=29320.0)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--long-ms", type=float, default=0.0)
    a = ap.parse_args(argv)
    if a.long_ms > 0:
        return _long(a)
    A = torch.empty(8192, 4096, device="cuda", dtype=torch.bfloat16)
    B = torch.empty(14336, 4096, device="cuda", dtype=torch.bfloat16)
    C = torch.empty(8192, 14336, device="cuda", dtype=torch.bfloat16)
    gemm.fill_random_(A, 1)
    gemm.fill_random_(B, 2)
    stamp = torch.zeros(8, dtype=torch.int64, device="cuda")
    kinds = {
        "idle_wait": lambda: gemm.idle_wait_us(a.us),
        "busy_spin": lambda: gemm.busy_spin_us(a.us),
        "gemm_deadline": lambda: gemm.gemm_deadline_us(A, B, C, a.us, stamp=stamp),
    }
    print(json.dumps({"wallclock_hz": _native.lib().dlnb_wallclock_hz(0)}))
    for name, fn in kinds.items():
        fn()
        torch.cuda.synchronize()
        ev = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            ev.append((e0, e1))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            fn()
        torch.cuda.synchronize()
        host_ms = (time.perf_counter() - t0) * 1e3 / a.reps
        ms = [e0.elapsed_time(e1) for e0, e1 in ev]
        med = statistics.median(ms)
        print(json.dumps({"kernel": name, "target_ms": a.us / 1e3, "event_ms_median": round(med, 4),
                          "event_rel_err": round(med / (a.us / 1e3) - 1, 5),
                          "host_ms_per_launch": round(host_ms, 4),
                          "host_rel_err": round(host_ms / (a.us / 1e3) - 1, 5)}), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
