"""Failure containment of the device-side machinery: a gate that is never raised inside a
lane-graph step (the compute program waits for it, and so does the pre-armed next replay's lane) must not
hold the GPU. The host's iteration timeout raises the device abort word - every device wait gives up - and
the CLI process ends at once (exit 3, no teardown: the driver reclaims its queues), so a fresh process right
after runs the same step at its floor."""
import os
import subprocess
import sys
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from dlnetbench_amd import engine  # noqa: E402


def _gpu():
    from dlnetbench_amd import _native
    try:
        return _native.lib().dlnb_gpu_count() > 0
    except Exception:  # noqa: BLE001
        return False


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not _gpu():
        pytest.skip("no GPU")


def _run(env_extra, runs=2, timeout=120):
    args = engine.build_args("fsdp", "llama3_8b_16_bfloat16", 32, 1, base_path=ROOT, warmup=1, runs=runs,
                             backend="rccl", graph=True, time_scale=0.05, json=None, quiet=True)
    env = dict(os.environ, DLNB_NO_TORCH="1", **env_extra)
    t0 = time.monotonic()
    p = subprocess.run([os.path.join(ROOT, "build", "bin", "fsdp"), *args], capture_output=True, text=True,
                       timeout=timeout, env=env)
    return p, time.monotonic() - t0


def _median(p):
    import json
    out = p.stdout
    b = out.index("<<<DLNB_REPORT_BEGIN")
    doc = json.loads(out[out.index("\n", b) + 1:out.index("<<<DLNB_REPORT_END")])
    it = doc["global"]["dlnb"]["iteration"]
    return doc, it["median_ms"], it["compute_floor_ms"]


def test_never_raised_gate_exits_fast_and_frees_the_gpu():
    """One lane-graph FSDP step of the headline config at 0.05x time whose first all-gather gate is never
    raised (DLNB_INJECT_FAULT mode=gate), with 60-s device gate waits and DLNB_TIMEOUT=5: the process exits
    with code 3 within 10 s of a normal run's time, saying the device waits were aborted; a fresh process
    started right after runs the step at its floor (no CUs still held)."""
    ok, t_ok = _run({})
    assert ok.returncode == 0, ok.stderr[-2000:]
    doc, med, floor = _median(ok)
    assert doc["global"]["dlnb"]["lane_graphs"]["enabled"], doc["global"]["dlnb"]["lane_graphs"]
    bad, t_bad = _run({"DLNB_INJECT_FAULT": "rank=0,iter=0,mode=gate", "DLNB_GATE_TIMEOUT_S": "60",
                       "DLNB_TIMEOUT": "5"})
    assert bad.returncode == 3, (bad.returncode, bad.stderr[-2000:])
    assert "device waits aborted" in bad.stderr, bad.stderr[-2000:]
    assert "gate signal 0 will not be raised" in bad.stderr
    # setup + the 5-s host timeout, not the 60-s device gate timeout
    assert t_bad <= t_ok + 10.0, (t_bad, t_ok)
    again, _ = _run({})
    assert again.returncode == 0, again.stderr[-2000:]
    _, med2, floor2 = _median(again)
    assert med2 <= floor2 * 1.02 + 0.5, (med2, floor2, med)


def test_library_host_recovers_after_a_device_failure():
    """The same failure in a library host (python, DLNB_FAIL_EXIT=0: nothing ends the process): the run
    raises, the device drains after the abort (nothing left spinning), and the next run in the same process
    completes at its floor."""
    code = r"""
import os, sys, json, time
sys.path.insert(0, %r)
os.environ["DLNB_NO_TORCH"] = "1"
from dlnetbench_amd import engine
kw = dict(base_path=%r, warmup=1, runs=2, backend="rccl", graph=True, time_scale=0.05, quiet=True)
os.environ.update(DLNB_INJECT_FAULT="rank=0,iter=0,mode=gate", DLNB_GATE_TIMEOUT_S="60", DLNB_TIMEOUT="5",
                  DLNB_FAIL_EXIT="0")
t0 = time.monotonic()
try:
    engine.run("fsdp", "llama3_8b_16_bfloat16", 32, 1, **kw)
    print("NO-ERROR")
except Exception as e:
    print("ERROR", time.monotonic() - t0, str(e)[:200])
del os.environ["DLNB_INJECT_FAULT"]
d = engine.run("fsdp", "llama3_8b_16_bfloat16", 32, 1, **kw)
it = d["global"]["dlnb"]["iteration"]
print("OK", json.dumps([it["median_ms"], it["compute_floor_ms"]]))
""" % (ROOT, ROOT)
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, DLNB_NO_TORCH="1"))
    assert p.returncode == 0, p.stderr[-3000:]
    lines = p.stdout.splitlines()
    err = [x for x in lines if x.startswith("ERROR")]
    assert err and "did not complete within DLNB_TIMEOUT" in err[0], p.stdout + p.stderr[-2000:]
    import json
    med, floor = json.loads([x for x in lines if x.startswith("OK")][0][3:])
    assert med <= floor * 1.02 + 0.5, (med, floor)
