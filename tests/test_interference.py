"""python -m dlnetbench_amd interference: a victim job alone and beside a
--loop aggressor (the reference's *_loop traffic generators, paired)."""
from __future__ import annotations

import os
import subprocess

import pytest

from dlnetbench_amd.tools import interference

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DATA = os.path.join(ROOT, "tests", "data")


def _no_leftover(name: str) -> bool:
    out = subprocess.run(["ps", "-eo", "args"], capture_output=True, text=True).stdout
    return not any(ln.startswith(os.path.join(ROOT, "build", "bin", name)) and "--loop" in ln
                   for ln in out.splitlines())


def test_victim_alone_then_beside_a_loop_aggressor():
    """2-rank FSDP victim, 2-rank DP aggressor (gpt2_l: 4 x 387 MB all-reduces per
    iteration over shared memory) on the shm backend: both phases report, the
    aggressor was running for the whole contended phase and is gone after."""
    r = interference.run(f"fsdp tiny_dense_8_bfloat16 4 2 {DATA} --backend cpu --compute sleep -w 1 -r 4", 2,
                         f"dp gpt2_l_16_bfloat16 4 {ROOT} --backend cpu --compute sleep", 2, warm_s=2.0,
                         timeout=120)
    for k in ("alone", "contended"):
        assert r[k]["world_size"] == 2 and r[k]["backend"] == "CPU-SHM"
        assert r[k]["median_ms"] >= 0.9 * r[k]["floor_ms"] > 0
    assert r["slowdown"] > 0 and r["aggressor"].endswith("--loop")
    assert set(r["comm"]) == {"allgather", "reduce_scatter"}
    assert all(c["alone_busbw_GBps"] > 0 and c["busbw_ratio"] > 0 for c in r["comm"].values())
    assert _no_leftover("dp")


def test_job_spec_needs_a_strategy():
    with pytest.raises(ValueError):
        interference._cmd("nonsense 1 2")


@pytest.mark.gpu
def test_interference_same_gpu():
    """Victim and aggressor on the one MI355X, each its own 1-rank RCCL job:
    the victim's fixed-work compute (gemm-work) shares the CUs with the
    aggressor's deadline GEMMs, so it cannot get faster."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    r = interference.run(f"fsdp tiny_dense_8_bfloat16 4 1 {DATA} --backend rccl --compute gemm-work -w 1 -r 2", 1,
                         f"dp tiny_dense_8_bfloat16 4 {DATA} --backend rccl --compute gemm", 1, warm_s=2.0,
                         timeout=120)
    assert r["alone"]["backend"] == "RCCL" and r["slowdown"] > 0.95, r
    assert r["fixed_work_cal"]  # the contended run reused the alone calibration (DLNB_FIXED_WORK_CAL)
    assert _no_leftover("dp")
