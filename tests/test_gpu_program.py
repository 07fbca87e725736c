"""The compute program kernel (kernels::gemm_tn_deadline_program) at kernel level: one
persistent launch running a list of tasks back to back, each with the start protocol of
csrc/kernels/deadline_sync.hpp - tile numerics, chained starts, late gates, done gates, the join, gate
timeouts, the host's abort word, blocks that come late for a task, and fixed-work tasks (their own start
and end stamps, the wait for the previous task on every block)."""
import time

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


from dlnetbench_amd import _native  # noqa: E402
from dlnetbench_amd.ops import gemm  # noqa: E402

MASK48 = (1 << 48) - 1
PROG_BIT = 1 << 63
# kernels::DlCounter
K_CAPPED, K_GATE_TIMEOUTS, K_ABORTED, K_LATE = 0, 3, 6, 7


def _hz():
    return _native.lib().dlnb_wallclock_hz(0)


def _ticks(us):
    return int(round(us * 1e-6 * _hz()))


def _grid():
    # leave 32 CUs free, as the runtime does: the other stream's one-wave kernels need room
    return torch.cuda.get_device_properties(0).multi_processor_count - 32


def _operands(dtype="bf16", M=512, N=512, K=4096, seed=1):
    g = torch.Generator(device="cuda").manual_seed(seed)
    a = torch.randn(M, K, device="cuda", generator=g)
    b = torch.randn(N, K, device="cuda", generator=g)
    if dtype == "fp8":
        if not hasattr(torch, "float8_e4m3fn"):
            pytest.skip("torch without float8")
        a, b = (a * 0.5).to(torch.float8_e4m3fn), (b * 0.5).to(torch.float8_e4m3fn)
    else:
        a, b = a.to(torch.bfloat16), b.to(torch.bfloat16)
    c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    return a, b, c


class Words:
    """An int64 CUDA tensor of device words and their addresses."""

    def __init__(self, n, fill=0):
        self.t = torch.full((n,), fill, dtype=torch.int64, device="cuda")

    def at(self, i):
        return self.t.data_ptr() + 8 * i

    def list(self):
        return [x & ((1 << 64) - 1) for x in self.t.tolist()]


def _task(**kw):
    t = _native.TaskDesc()
    for k, v in kw.items():
        setattr(t, k, v)
    return t


def _buf(n):
    return torch.zeros(n * gemm.task_size(), dtype=torch.uint8, device="cuda")


def _assert_close(c, ref):
    err = (c.float() - ref).abs()
    bound = ref.abs() * 2.0 ** -8 + 1e-3 * ref.pow(2).mean().sqrt().item()
    assert (err - bound).max().item() <= 0, (err.max().item(), ref.pow(2).mean().sqrt().item())


@pytest.mark.parametrize("dtype,bf16_kernel", [("bf16", "8phase"), ("bf16", "4wave"), ("fp8", "8phase"),
                                               ("bf16_oddk", "8phase"), ("fp8_k384", "8phase")])
def test_program_tiles_match_torch(dtype, bf16_kernel, monkeypatch):
    """Every C tile equals A.B^T against fp32 torch after a 5-task program (C NaN-poisoned first): the
    program kernels (8-phase bf16 balanced / plain, one-wave-per-SIMD bf16 and fp8 MX, 8-phase fp8) store
    complete tiles only, task after task."""
    monkeypatch.setenv("DLNB_DEADLINE_BF16", bf16_kernel)
    K = {"bf16_oddk": 1216, "fp8_k384": 384}.get(dtype, 4096)
    a, b, c = _operands(dtype.split("_")[0], K=K, seed=K)
    assert gemm.program_ktiles(512, 512, K, a.dtype) > 0
    slot, it = Words(8), Words(1, 3)
    tasks = [_task(ticks=_ticks(700.0), chain_ticks=_ticks(30.0) if k else 0, epoch=k) for k in range(5)]
    gemm.gemm_program(a, b, c, tasks, slot.t, _buf(5), iter_word=it.t, grid=_grid())
    torch.cuda.synchronize()
    assert not torch.isnan(c.float()).any(), "some tile was never stored"
    _assert_close(c, a.float() @ b.float().t())


def test_program_chained_starts():
    """Chained program tasks start exactly at the previous task's deadline: t[k+1] = t[k] + ticks[k]
    (+-1 tick) - no kernel boundary between them to absorb - and the program lasts their sum."""
    a, b, c = _operands(K=4096)
    slot, it, ts, counters = Words(8), Words(1), Words(8), Words(8)
    durs = [800.0, 1500.0, 300.0, 2000.0, 600.0]
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for rep in range(2):  # the first round also loads the kernel
        it.t.fill_(rep + 1)
        tasks = [_task(ticks=_ticks(u), chain_ticks=_ticks(30.0) if k else 0, epoch=k, tstart0=ts.at(k))
                 for k, u in enumerate(durs)]
        e0.record(s)
        gemm.gemm_program(a, b, c, tasks, slot.t, _buf(5), iter_word=it.t, counters=counters.t, grid=_grid())
        e1.record(s)
        torch.cuda.synchronize()
    t = ts.list()
    for k in range(4):
        assert abs(t[k + 1] - t[k] - _ticks(durs[k])) <= 1, (k, t)
    ms = e0.elapsed_time(e1)
    assert sum(durs) / 1e3 <= ms * 1.005 and ms <= sum(durs) / 1e3 * 1.01 + 0.1, ms
    assert counters.list()[K_CAPPED] == 0


def test_program_gated_task_starts_at_late_gate():
    """A gated program task whose gate is raised (on another stream, 3 ms after the program began) after the
    previous task's deadline starts at the gate's time - the wait is exposed, never absorbed - and the next
    chained task at its deadline from there."""
    a, b, c = _operands()
    slot, it, ts, gates = Words(8), Words(1), Words(8), Words(4)
    other = torch.cuda.Stream()
    s = torch.cuda.current_stream()
    for rep in range(2):
        it.t.fill_(10 + rep)
        tag = 5 + rep
        e0 = torch.cuda.Event()
        e0.record(s)
        torch.cuda.synchronize()
        with torch.cuda.stream(other):
            gemm.idle_wait_us(3000.0)
            gemm.gate_signal_iter_(gates.t, 0, tag, it.t)
        tasks = [_task(ticks=_ticks(1000.0), epoch=0, tstart0=ts.at(0)),
                 _task(ticks=_ticks(1000.0), chain_ticks=_ticks(30.0), epoch=1, tstart0=ts.at(1),
                       gate0=gates.at(0), tag0=tag),
                 _task(ticks=_ticks(500.0), chain_ticks=_ticks(30.0), epoch=2, tstart0=ts.at(2))]
        gemm.gemm_program(a, b, c, tasks, slot.t, _buf(3), iter_word=it.t, grid=_grid())
        torch.cuda.synchronize()
    g, t = gates.list(), ts.list()
    assert g[0] == (11 << 32) | 6, g  # seq = iteration << 32 | tag
    assert (t[1] & MASK48) == (g[1] & MASK48), (t, g)  # started at the late gate
    assert t[1] - t[0] >= _ticks(1000.0) + _ticks(500.0), t  # well after task 0's deadline
    assert abs(t[2] - t[1] - _ticks(1000.0)) <= 1, t


@pytest.mark.parametrize("fixed", [False, True])
def test_program_gate_only_task(fixed):
    """A gate-only task (flags = 1: a stream's event wait and record folded into its compute program) between
    two tasks, its gate raised on another stream 3 ms after the program began: no tiles, its done gate up
    within 20 us of its gate, and the next task starts there - a chained deadline task continues from when
    the gates opened, a fixed-work task once the gate-only task is complete on every block."""
    a, b, c = _operands()
    slot, it, ts, gates, done, te = Words(8), Words(1), Words(8), Words(4), Words(4), Words(8)
    other = torch.cuda.Stream()
    s = torch.cuda.current_stream()
    for rep in range(2):
        it.t.fill_(20 + rep)
        tag = 9 + rep
        e0 = torch.cuda.Event()
        e0.record(s)
        torch.cuda.synchronize()
        with torch.cuda.stream(other):
            gemm.idle_wait_us(3000.0)
            gemm.gate_signal_iter_(gates.t, 0, tag, it.t)
        if fixed:
            work = dict(ticks=0, work_rounds=1)
            tasks = [_task(epoch=0, tstart0=ts.at(0), tend=te.at(0), **work),
                     _task(ticks=0, flags=1, epoch=1, gate0=gates.at(0), tag0=tag, done_gate=done.at(0),
                           done_tag=50, tstart0=ts.at(1)),
                     _task(epoch=2, tstart0=ts.at(2), tend=te.at(2), **work)]
        else:
            tasks = [_task(ticks=_ticks(1000.0), epoch=0, tstart0=ts.at(0)),
                     _task(ticks=1, flags=1, epoch=1, gate0=gates.at(0), tag0=tag, done_gate=done.at(0),
                           done_tag=50, tstart0=ts.at(1)),
                     _task(ticks=_ticks(500.0), chain_ticks=_ticks(30.0), epoch=2, tstart0=ts.at(2))]
        gemm.gemm_program(a, b, c, tasks, slot.t, _buf(3), iter_word=it.t, grid=_grid())
        torch.cuda.synchronize()
    g, t, d = gates.list(), ts.list(), done.list()
    assert d[0] == (21 << 32) | 50, d  # the gate-only task's done gate, this iteration's sequence
    gate_t = g[1] & MASK48
    us = lambda x: x / _hz() * 1e6  # noqa: E731
    assert 0 <= us((t[1] & MASK48) - gate_t) <= 20.0, (t, g)  # it started when its gate opened
    assert 0 <= us((d[1] & MASK48) - gate_t) <= 20.0, (d, g)
    assert 0 <= us((t[2] & MASK48) - gate_t) <= 20.0, (t, g)  # the next task right behind it
    if not fixed:
        assert t[1] - t[0] >= _ticks(1000.0) + _ticks(500.0), t


def test_program_done_gates_at_deadlines():
    """Each task's done gate is raised by block 0 as it leaves the task: within 20 us after the task's
    deadline (start + ticks), carrying the iteration's sequence."""
    a, b, c = _operands()
    slot, it, ts, done = Words(8), Words(1, 7), Words(8), Words(16)
    durs = [600.0, 900.0, 400.0, 1200.0]
    for rep in range(2):
        tasks = [_task(ticks=_ticks(u), chain_ticks=_ticks(30.0) if k else 0, epoch=k, tstart0=ts.at(k),
                       done_gate=done.at(2 * k), done_tag=100 + k) for k, u in enumerate(durs)]
        it.t.fill_(7 + rep)
        gemm.gemm_program(a, b, c, tasks, slot.t, _buf(4), iter_word=it.t, grid=_grid())
        torch.cuda.synchronize()
    t, d = ts.list(), done.list()
    for k, u in enumerate(durs):
        assert d[2 * k] == (8 << 32) | (100 + k), d
        late = (d[2 * k + 1] - (t[k] + _ticks(u))) / _hz() * 1e6
        assert 0 <= late <= 20.0, (k, late)


def test_program_join_after_end_gates():
    """The join (the program's last task) stores the iteration into its done word only after its gates are
    up: here a gate raised 4 ms after the program's last compute task ended, so the join's time stamp is at
    or after the gate's."""
    a, b, c = _operands()
    slot, it, gates = Words(8), Words(1, 21), Words(4)
    done, tj = Words(1, -1), Words(1)
    other = torch.cuda.Stream()
    s = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(s)
    torch.cuda.synchronize()
    with torch.cuda.stream(other):
        gemm.idle_wait_us(5000.0)
        gemm.gate_signal_iter_(gates.t, 0, 3, it.t)
    tasks = [_task(ticks=_ticks(1000.0), epoch=0), _task(epoch=1, gate0=gates.at(0), tag0=3, tstart0=done.at(0),
                                                         tstart1=tj.at(0))]
    gemm.gemm_program(a, b, c, tasks, slot.t, _buf(2), iter_word=it.t, grid=_grid())
    torch.cuda.synchronize()
    assert done.list()[0] == 21
    g = gates.list()
    assert tj.list()[0] >= g[1], (tj.list(), g)


def test_program_join_of_several_tasks():
    """Three end gates (four lanes) make the join two tasks - two gates, then one gate and the host's done word:
    every one of them runs (the kernel returned after the first before round 6, so the done word never came and
    the host waited out its timeout), the done word only after the last gate (raised 3 ms late)."""
    a, b, c = _operands()
    slot, it, gates = Words(8), Words(1, 33), Words(8)
    done, tj = Words(1, -1), Words(1)
    other = torch.cuda.Stream()
    s = torch.cuda.current_stream()
    ev = torch.cuda.Event()
    ev.record(s)
    torch.cuda.synchronize()
    with torch.cuda.stream(other):
        gemm.gate_signal_iter_(gates.t, 0, 1, it.t)  # (gate index i: 16 bytes each - Words.at(2 i))
        gemm.gate_signal_iter_(gates.t, 1, 1, it.t)
        gemm.idle_wait_us(3000.0)
        gemm.gate_signal_iter_(gates.t, 2, 1, it.t)
    tasks = [_task(ticks=_ticks(500.0), epoch=0),
             _task(epoch=1, gate0=gates.at(0), tag0=1, gate1=gates.at(2), tag1=1),
             _task(epoch=2, gate0=gates.at(4), tag0=1, tstart0=done.at(0), tstart1=tj.at(0))]
    gemm.gemm_program(a, b, c, tasks, slot.t, _buf(3), iter_word=it.t, grid=_grid())
    torch.cuda.synchronize()
    assert done.list()[0] == 33, done.list()
    g = gates.list()
    assert tj.list()[0] >= g[5], (tj.list(), g)


def test_program_gate_timeout_counted():
    """A gate never raised ends the wait at the gate timeout (2 ms here): the task runs, kGateTimeouts counts
    it, and the program finishes."""
    a, b, c = _operands()
    slot, it, gates, counters = Words(8), Words(1, 2), Words(4), Words(8)
    tasks = [_task(ticks=_ticks(500.0), epoch=0, gate0=gates.at(0), tag0=9)]
    t0 = time.monotonic()
    gemm.gemm_program(a, b, c, tasks, slot.t, _buf(1), iter_word=it.t, counters=counters.t, gate_timeout_s=0.002,
                      grid=_grid())
    torch.cuda.synchronize()
    assert time.monotonic() - t0 < 5.0
    assert counters.list()[K_GATE_TIMEOUTS] == 1, counters.list()


def test_program_abort_word_ends_waits():
    """a program task gated on a gate that is never raised, with a 60-s gate timeout, leaves
    its wait as soon as the host raises the abort word (the claimer and every block waiting for its publish),
    ends its deadline task at once and counts kAborted - the kernel drains in well under a second instead of
    holding the CUs for the timeout."""
    a, b, c = _operands()
    slot, it, gates, counters = Words(8), Words(1, 4), Words(4), Words(8)
    abort = gemm.HostWords(1)
    try:
        tasks = [_task(ticks=_ticks(30000.0), epoch=0, gate0=gates.at(0), tag0=1),
                 _task(ticks=_ticks(30000.0), chain_ticks=_ticks(30.0), epoch=1, gate0=gates.at(2), tag0=1)]
        gemm.gemm_program(a, b, c, tasks, slot.t, _buf(2), iter_word=it.t, counters=counters.t, abort=abort,
                          gate_timeout_s=60.0, grid=_grid())
        time.sleep(0.2)
        t0 = time.monotonic()
        abort[0] = 1
        torch.cuda.synchronize()
        drained = time.monotonic() - t0
        v = counters.list()
    finally:
        abort.free()
    assert drained < 1.0, drained
    assert v[K_ABORTED] >= 2 and v[K_GATE_TIMEOUTS] == 0, v


def test_program_late_blocks_skip_overtaken_tasks():
    """program claims are monotonic (iteration * 4096 + task). A block that reaches a task after a
    later task was claimed skips it instead of claiming it back: here the slot already carries a later claim,
    so every block of every task is late - each deadline task ends at once (kLateBlocks = grid x tasks) and
    the 2-s tasks take no time."""
    a, b, c = _operands()
    slot, it, counters = Words(8), Words(1, 50), Words(8)
    slot.t[2] = (PROG_BIT | (51 * 4096)) - (1 << 64)  # a claim of iteration 51 (int64 view)
    tasks = [_task(ticks=_ticks(2e6), chain_ticks=_ticks(30.0) if k else 0, epoch=k) for k in range(3)]
    t0 = time.monotonic()
    gemm.gemm_program(a, b, c, tasks, slot.t, _buf(3), iter_word=it.t, counters=counters.t, grid=_grid())
    torch.cuda.synchronize()
    assert time.monotonic() - t0 < 1.0  # three 2-s tasks, all skipped
    assert counters.list()[K_LATE] == 3 * _grid(), counters.list()


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_program_fixed_work_task(dtype):
    """A fixed-work task launched on its own (one-task program with a launch epoch): every block computes
    `rounds` full tiles - every C tile equals A.B^T - its claimer stamps the start, the block that completes the
    task on the whole grid stamps the end and raises the done gate at that time, and the slot's completion
    count is a multiple of the grid."""
    a, b, c = _operands(dtype)
    slot, ts, te, done = Words(8), Words(2), Words(2), Words(2)
    task = _task(work_rounds=3, epoch=0, tstart0=ts.at(0), tend=te.at(0), done_gate=done.at(0), done_tag=4)
    gemm.gemm_program(a, b, c, [task], slot.t, _buf(1), grid=_grid(), epoch=40000)
    torch.cuda.synchronize()
    assert not torch.isnan(c.float()).any()
    _assert_close(c, a.float() @ b.float().t())
    t0, t1, d = ts.list()[0], te.list()[0], done.list()
    assert t1 > t0 and d[0] == 4 and d[1] == t1, (t0, t1, d)
    assert slot.list()[3] % _grid() == 0 and slot.list()[3] > 0, slot.list()


def test_program_fixed_work_waits_for_previous_task():
    """Fixed-work tasks in one program: task k+1 starts only once task k is complete on every block
    (start[k+1] >= end[k]); each lasts about its work (a tail tile of half the K-tiles adds about half a
    round), and twice the work takes about twice as long."""
    a, b, c = _operands(M=4096, N=4096, K=4096)
    nk = gemm.program_ktiles(4096, 4096, 4096, a.dtype)
    slot, it, ts, te = Words(8), Words(1), Words(8), Words(8)
    work = [(4, 0), (8, 0), (4, nk // 2), (2, 0)]
    for rep in range(2):
        it.t.fill_(rep + 1)
        tasks = [_task(work_rounds=r, tail_kt=tk, epoch=k, tstart0=ts.at(k), tend=te.at(k))
                 for k, (r, tk) in enumerate(work)]
        gemm.gemm_program(a, b, c, tasks, slot.t, _buf(4), iter_word=it.t, grid=_grid())
        torch.cuda.synchronize()
    t, e = ts.list(), te.list()
    dur = [e[k] - t[k] for k in range(4)]
    for k in range(3):
        assert t[k + 1] >= e[k], (k, t, e)
    assert all(x > 0 for x in dur), dur
    assert 1.6 <= dur[1] / dur[0] <= 2.4, dur
    assert 1.05 <= dur[2] / dur[0] <= 1.4, dur
