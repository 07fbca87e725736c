"""The remaining tool front ends: rocprofv3 summaries and the offline model-config
cache on CPU; the GEMM benchmark and the deadline clock check on the GPU."""
from __future__ import annotations

import json
import os

import pytest

from dlnetbench_amd.tools import download_models, prof_summary


def test_prof_summary_kernel_stats(tmp_path, capsys):
    """rocprofv3 --stats CSV -> markdown table (names shortened, template args kept)."""
    d = tmp_path / "prof"
    d.mkdir()
    (d / "x_kernel_stats.csv").write_text(
        "Name,Calls,TotalDurationNs,AverageNs,Percentage,MinNs,MaxNs,StdDev\n"
        "\"void dlnb::kernels::gemm_8phase_kernel<false, true, true, false>(dlnb::kernels::Args)\",128,"
        "5630020000,43984531.2,31.15,1,2,0\n"
        "dlnb::kernels::stamp_kernel(unsigned long*),6666,120130000,18021.3,0.66,1,2,0\n")
    md = prof_summary.kernel_stats(str(d))
    lines = md.splitlines()
    assert lines[0].startswith("| kernel | calls") and len(lines) == 4
    assert "`void dlnb::kernels::gemm_8phase_kernel<false, true, true, false>` | 128 | 5630.02 | 43984.5 | 31.15" in md
    assert "`dlnb::kernels::stamp_kernel` | 6666 | 120.13 | 18.0 | 0.66" in md


def test_download_models_offline(tmp_path, capsys):
    """No network on the target image: --list prints the registry, and a
    model's config is written from the shipped architecture JSON."""
    assert download_models.main(["--list"]) == 0
    out = capsys.readouterr().out
    assert "llama3_8b" in out and "meta-llama/Meta-Llama-3-8B" in out
    assert download_models.main(["llama3_8b", "--cache", str(tmp_path)]) == 0
    cfg = tmp_path / "meta-llama--Meta-Llama-3-8B" / "config.json"
    assert cfg.exists() and json.loads(cfg.read_text())


@pytest.mark.gpu
def test_gemm_bench_and_clock_check(capsys):
    """gemm_bench: one small shape, ours next to hipBLASLt; clock_check: the
    deadline kernels (idle, spin, GEMM) land on a 2 ms target."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from dlnetbench_amd.tools import clock_check, gemm_bench
    assert gemm_bench.main(["--shapes", "2048x2048x2048", "--rounds", "2", "--iters", "3"]) == 0
    rows = [json.loads(ln) for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    assert rows and rows[0]["M"] == 2048 and rows[0]["v0_tflops_median"] > 50 and rows[0]["torch_tflops_median"] > 50
    assert clock_check.main(["--us", "2000", "--reps", "3"]) == 0
    rows = [json.loads(ln) for ln in capsys.readouterr().out.splitlines() if ln.startswith("{")]
    kinds = {r["kernel"]: r for r in rows if "kernel" in r}
    assert set(kinds) == {"idle_wait", "busy_spin", "gemm_deadline"}
    for r in kinds.values():
        assert abs(r["event_rel_err"]) < 0.05, r
