"""Numerics of the hand-written gfx950 kernels against fp32 PyTorch references."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


from dlnetbench_amd.ops import gemm  # noqa: E402


def assert_close_bf16_out(c, ref):
    """fp32-accumulated GEMM with a bf16 output: every element within one bf16
    rounding of the fp32 reference (2^-8 relative) plus 1e-3 of the RMS of the
    reference for accumulation-order differences. A dropped or doubled K tile
    moves elements by O(rms) and fails this."""
    err = (c.float() - ref).abs()
    bound = ref.abs() * 2.0 ** -8 + 1e-3 * ref.pow(2).mean().sqrt().item()
    worst = (err - bound).max().item()
    assert worst <= 0, f"max excess {worst}, max err {err.max().item()}, rms {ref.pow(2).mean().sqrt().item()}"


# gemm_tn variants (kernels.hpp): 0 default (bf16: narrow tiles when square ones leave CUs idle), 5 4-wave (MX fp8,
# or bf16 two 16x16x32 MFMAs per K-tile row; K % 128 == 0, else it falls through to 6), 6 8-phase, 8 8-wave
@pytest.mark.parametrize("waves", [0, 5, 6, 8])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (256, 512, 128), (512, 512, 64), (768, 256, 128),
                                   (512, 256, 1024), (768, 1280, 640), (2048, 1024, 4096), (256, 256, 192),
                                   (512, 768, 320)])
def test_gemm_bf16_matches_torch(M, N, K, waves):
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
    c = gemm.gemm_tn(a, b, waves=waves)
    torch.cuda.synchronize()
    assert_close_bf16_out(c, a.float() @ b.float().t())


@pytest.mark.parametrize("waves", [0, 6, 8])
def test_gemm_bf16_identity_asymmetric(waves):
    # A = I picks rows of B: catches any row/column/quadrant swap in the C write.
    M = N = 256
    K = 256
    a = torch.eye(M, K, device="cuda", dtype=torch.bfloat16)
    b = (torch.arange(N * K, device="cuda", dtype=torch.float32).reshape(N, K) % 97 / 8.0).to(torch.bfloat16)
    c = gemm.gemm_tn(a, b, waves=waves)
    torch.cuda.synchronize()
    assert torch.equal(c.float(), b.float().t())


@pytest.mark.skipif(not hasattr(torch, "float8_e4m3fn"), reason="torch without float8")
@pytest.mark.parametrize("waves", [0, 6])
@pytest.mark.parametrize("M,N,K", [(256, 256, 128), (512, 256, 128), (256, 512, 256), (512, 768, 512),
                                   (1024, 512, 2048), (512, 512, 384)])
def test_gemm_fp8_matches_torch(M, N, K, waves):
    g = torch.Generator(device="cuda").manual_seed(7 + M)
    a = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.float8_e4m3fn)
    b = (torch.randn(N, K, device="cuda", generator=g) * 0.5).to(torch.float8_e4m3fn)
    c = gemm.gemm_tn(a, b, waves=waves)
    torch.cuda.synchronize()
    assert_close_bf16_out(c, a.float() @ b.float().t())


@pytest.mark.parametrize("M,N,K,nf", [(2048, 1280, 128, 4), (8192, 1280, 5120, 5), (7168, 1280, 640, 5),
                                      (8192, 1536, 256, 6), (512, 768, 1024, 3), (8192, 768, 3072, 3),
                                      (8192, 5120, 256, 5), (8192, 3072, 384, 6), (8192, 1792, 6400, 7)])
def test_gemm_bf16_narrow_tiles(M, N, K, nf):
    """bf16 through the narrow-tile kernel (two 16x16x32 MFMAs per 128-byte K-tile row on the MX kernel's
    fragments), K down to the 2-K-tile minimum."""
    from dlnetbench_amd import _native
    assert _native.lib().dlnb_gemm_narrow_nf(M, N, torch.cuda.get_device_properties(0).multi_processor_count) == nf
    g = torch.Generator(device="cuda").manual_seed(M + N + K + nf)
    a = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    b = torch.randn(N, K, device="cuda", generator=g).to(torch.bfloat16)
    c = gemm.gemm_tn(a, b)
    torch.cuda.synchronize()
    assert_close_bf16_out(c, a.float() @ b.float().t())


@pytest.mark.skipif(not hasattr(torch, "float8_e4m3fn"), reason="torch without float8")
@pytest.mark.parametrize("M,N,K,nf", [(2048, 1280, 256, 4), (8192, 1280, 5120, 5), (7168, 1280, 512, 5),
                                      (8192, 1536, 256, 6), (8192, 1024, 1280, 4), (768, 512, 2048, 4),
                                      (8192, 768, 3072, 3), (2048, 768, 256, 3), (8192, 5120, 512, 5),
                                      (8192, 3072, 256, 6), (8192, 1792, 6400, 7), (2048, 1792, 256, 4)])
def test_gemm_fp8_narrow_tiles(M, N, K, nf):
    """Fewer 256 x 256 tiles than CUs, or a partial last round (8192 x 5120: 640 square tiles): the MX fp8
    kernel's 256 x 32 nf tiles (gemm_4wave_fp8.hip, narrow kernel), including the ViT-H FFN down projection
    8192 x 1280 x 5120 (the C5 stand-in shape) and the 2-K-tile minimum."""
    from dlnetbench_amd import _native
    assert _native.lib().dlnb_gemm_narrow_nf(M, N, torch.cuda.get_device_properties(0).multi_processor_count) == nf
    g = torch.Generator(device="cuda").manual_seed(M + N + K + nf)
    a = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.float8_e4m3fn)
    b = (torch.randn(N, K, device="cuda", generator=g) * 0.5).to(torch.float8_e4m3fn)
    c = gemm.gemm_tn(a, b)
    torch.cuda.synchronize()
    assert_close_bf16_out(c, a.float() @ b.float().t())


@pytest.mark.skipif(not hasattr(torch, "float8_e4m3fn"), reason="torch without float8")
@pytest.mark.parametrize("M,N,K", [(4096, 4352, 512), (8192, 8192, 256), (2048, 8448, 1280), (6144, 2048, 256)])
def test_gemm_fp8_many_tiles(M, N, K):
    """More tiles than CUs: the one-wave-per-SIMD fp8 kernel runs as the streaming persistent kernel (a
    block's tiles as one K-tile stream, the next tile's first K-tiles staged during the current one's
    last, K = 256 the 2-K-tile minimum); fewer tiles (test_gemm_fp8_matches_torch) a block per tile - square
    tiles where no narrower one saves a round (6144 x 2048: 192 tiles), else test_gemm_fp8_narrow_tiles."""
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = (torch.randn(M, K, device="cuda", generator=g) * 0.5).to(torch.float8_e4m3fn)
    b = (torch.randn(N, K, device="cuda", generator=g) * 0.5).to(torch.float8_e4m3fn)
    c = gemm.gemm_tn(a, b)
    torch.cuda.synchronize()
    assert_close_bf16_out(c, a.float() @ b.float().t())


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("M,N,Kb", [(512, 512, 256), (512, 768, 512), (768, 512, 768), (1024, 512, 1024),
                                    (512, 512, 5120), (8192, 8192, 512), (4096, 4352, 1280), (6144, 4096, 2048)])
def test_gemm_4wave_k_tile_counts(M, N, Kb, dtype, monkeypatch):
    """The one-wave-per-SIMD square kernels' K-loop split (gemm_4wave_fp8.hip ktiles_rest: clamp-free main
    pairs, then the general last pair and K-tile): K from the 2-K-tile minimum (no main-loop pair) through 4
    (the last pair only), 6, 8 and 40 K-tiles; fewer tiles than CUs (a block per tile) and more (the streaming
    kernel, whose last K-tiles stage the next tile's). Kb = K in bytes."""
    if dtype == "fp8" and not hasattr(torch, "float8_e4m3fn"):
        pytest.skip("torch without float8")
    monkeypatch.setenv("DLNB_GEMM_NARROW_NF", "8")  # square tiles only: this test is about those kernels
    K = Kb // 2 if dtype == "bf16" else Kb
    g = torch.Generator(device="cuda").manual_seed(M + N + K)
    a = torch.randn(M, K, device="cuda", generator=g) * 0.5
    b = torch.randn(N, K, device="cuda", generator=g) * 0.5
    dt = torch.bfloat16 if dtype == "bf16" else torch.float8_e4m3fn
    a, b = a.to(dt), b.to(dt)
    c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    gemm.gemm_tn(a, b, c, waves=5)
    torch.cuda.synchronize()
    assert_close_bf16_out(c, a.float() @ b.float().t())


@pytest.mark.parametrize("cpad", [256, 4])
@pytest.mark.parametrize("dtype,waves", [("bf16", 0), ("bf16", 6), ("bf16", 8), ("fp8", 0), ("fp8", 6), ("fp8", 8)])
def test_gemm_strided_operands(dtype, waves, cpad):
    """Row-strided A, B and C (views of wider matrices: leading dimensions > K, > N): the staging lane
    offsets and buffer resources use the leading dimensions, not K. cpad = 4: C rows only 8-byte aligned, so the
    epilogue keeps its 8-byte stores instead of the paired 16-byte ones (store_pair.hpp)."""
    if dtype == "fp8" and not hasattr(torch, "float8_e4m3fn"):
        pytest.skip("torch without float8")
    M, N, K = 512, 768, 512
    g = torch.Generator(device="cuda").manual_seed(11)
    A = torch.randn(M, K + 320, device="cuda", generator=g) * 0.5
    B = torch.randn(N, K + 192, device="cuda", generator=g) * 0.5
    if dtype == "fp8":
        A, B = A.to(torch.float8_e4m3fn), B.to(torch.float8_e4m3fn)
    else:
        A, B = A.to(torch.bfloat16), B.to(torch.bfloat16)
    a, b = A[:, 64:64 + K], B[:, 128:128 + K]
    Cbig = torch.full((M, N + cpad), float("nan"), device="cuda", dtype=torch.bfloat16)
    c = Cbig[:, :N]
    gemm.gemm_tn(a, b, c, waves=waves)
    torch.cuda.synchronize()
    assert_close_bf16_out(c, a.float() @ b.float().t())
    assert torch.isnan(Cbig[:, N:].float()).all(), "wrote outside C"


def test_fill_random_uniform():
    t = torch.empty(1 << 20, device="cuda", dtype=torch.bfloat16)
    gemm.fill_random_(t, seed=3)
    torch.cuda.synchronize()
    f = t.float()
    assert f.min().item() >= -1.0 and f.max().item() <= 1.0
    assert abs(f.mean().item()) < 0.01
    assert abs(f.std().item() - (1 / 3) ** 0.5) < 0.02


def test_sgd_momentum_matches_torch():
    n = 100003
    p = torch.randn(n, device="cuda").to(torch.bfloat16)
    m = torch.randn(n, device="cuda").to(torch.bfloat16)
    g = torch.randn(n, device="cuda").to(torch.bfloat16)
    m_ref = 0.9 * m.float() + g.float()
    p_ref = p.float() - 1e-2 * m_ref
    gemm.sgd_momentum_(p, m, g, lr=1e-2, beta=0.9)
    torch.cuda.synchronize()
    assert (m.float() - m_ref).abs().max().item() < 2e-2
    assert (p.float() - p_ref).abs().max().item() < 2e-2


@pytest.mark.parametrize("fn", ["idle", "spin"])
def test_deadline_kernels_hit_duration(fn):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    run = gemm.idle_wait_us if fn == "idle" else gemm.busy_spin_us
    run(50.0)  # first launch of the kernel (code object load) outside the timing
    torch.cuda.synchronize()
    for us in (200.0, 5000.0):
        times = []
        for _ in range(3):
            e0.record(s)
            run(us)
            e1.record(s)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        ms = sorted(times)[1]
        assert us / 1e3 * 0.97 <= ms <= us / 1e3 * 1.10 + 0.05, (us, times)


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
@pytest.mark.parametrize("us", [100.0, 2000.0, 30000.0])
def test_deadline_gemm_duration(us, dtype):
    a = torch.empty(8192, 4096, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(14336, 4096, device="cuda", dtype=torch.bfloat16)
    gemm.fill_random_(a, 1)
    gemm.fill_random_(b, 2)
    if dtype == "fp8":
        a, b = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
    c = torch.empty(8192, 14336, device="cuda", dtype=torch.bfloat16)
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    stamp = torch.zeros(8, dtype=torch.int64, device="cuda")
    for _ in range(3):  # warm: code object load, clocks out of idle
        gemm.gemm_deadline_us(a, b, c, us, stamp)
    times = []
    for _ in range(5):
        e0.record(s)
        gemm.gemm_deadline_us(a, b, c, us, stamp)
        e1.record(s)
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    ms = sorted(times)[2]
    assert us / 1e3 <= ms * 1.01 and ms <= us / 1e3 * 1.05 + 0.03, (us, times)


# (dtype, M, N, K, grid) -> the deadline kernel the shape selects (kernels.hip gemm_tn_deadline)
DEADLINE_CASES = [
    ("bf16", 1024, 768, 512, 3),   # <= 16 K-tiles: the streaming 8-phase kernel
    ("bf16", 512, 512, 256, 1),
    ("bf16", 256, 256, 256, 2),
    ("bf16", 768, 512, 1280, 0),   # 20 K-tiles: the per-tile loop, balanced reads
    ("bf16", 512, 512, 1216, 2),   # 19 K-tiles (odd): the per-tile loop, plain reads
    ("bf16", 256, 512, 64, 2),     # 1 K-tile: the 8-wave kernel
    ("fp8", 1024, 768, 512, 3),    # K % 256 == 0: the one-wave-per-SIMD MX kernel
    ("fp8", 512, 512, 256, 1),
    ("fp8", 768, 512, 1280, 0),
    ("fp8", 512, 768, 384, 2),     # K % 256 != 0: the 8-phase kernel, uniform K-tile body
    ("fp8", 768, 512, 640, 0),
    ("fp8", 256, 512, 128, 2),     # 1 K-tile: the 8-wave kernel
]


@pytest.mark.parametrize("bf16_kernel", ["8phase", "4wave"])
@pytest.mark.parametrize("dtype,M,N,K,grid", DEADLINE_CASES)
def test_deadline_gemm_numerics(M, N, K, grid, dtype, bf16_kernel, monkeypatch):
    """The persistent deadline GEMM (the bench's compute), every kernel the shapes select. With a deadline
    long enough for several passes every tile of C holds a complete product: each one equals A.B^T.
    Small grids make every block cross many tile boundaries (grid 0 = the default, CUs - 32)."""
    if dtype == "fp8" and not hasattr(torch, "float8_e4m3fn"):
        pytest.skip("torch without float8")
    if bf16_kernel == "4wave" and (dtype != "bf16" or K % 128):
        pytest.skip("the bf16 one-wave-per-SIMD deadline kernel: bf16, K % 128 == 0")
    monkeypatch.setenv("DLNB_DEADLINE_BF16", bf16_kernel)
    g = torch.Generator(device="cuda").manual_seed(M * 3 + N + K)
    a = torch.randn(M, K, device="cuda", generator=g)
    b = torch.randn(N, K, device="cuda", generator=g)
    if dtype == "fp8":
        a, b = (a * 0.5).to(torch.float8_e4m3fn), (b * 0.5).to(torch.float8_e4m3fn)
    else:
        a, b = a.to(torch.bfloat16), b.to(torch.bfloat16)
    c = torch.full((M, N), float("nan"), device="cuda", dtype=torch.bfloat16)
    stamp = torch.zeros(8, dtype=torch.int64, device="cuda")
    gemm.gemm_deadline_us(a, b, c, 3000.0, stamp, grid=grid)
    torch.cuda.synchronize()
    assert not torch.isnan(c.float()).any(), "some tile was never stored"
    assert_close_bf16_out(c, a.float() @ b.float().t())


def _grid():
    # leave 32 CUs free, as the runtime does: the gate / idle kernels of the other stream need room
    return torch.cuda.get_device_properties(0).multi_processor_count - 32


def _deadline_operands(dtype="bf16"):
    a = torch.empty(8192, 4096, device="cuda", dtype=torch.bfloat16)
    b = torch.empty(4096, 4096, device="cuda", dtype=torch.bfloat16)
    gemm.fill_random_(a, 1)
    gemm.fill_random_(b, 2)
    c = torch.empty(8192, 4096, device="cuda", dtype=torch.bfloat16)
    return a, b, c


@pytest.mark.parametrize("dtype", ["bf16", "fp8"])
def test_deadline_chain_continues_previous_deadline(dtype):
    """Chained deadline tasks (deadline_sync.hpp): a task that follows the previous one with only a launch hop
    starts exactly at its deadline (start stamp = previous start + ticks), so the hop is absorbed and the pair
    lasts the sum of their durations; a longer delay (here a 0.3 ms idle kernel between them, standing for a
    node queued in between) is absorbed only up to the chain's cap (30 us): the task starts 30 us before its
    first block arrived and the rest stays in the elapsed time. An unchained task starts when its first block
    arrives."""
    a, b, c = _deadline_operands()
    if dtype == "fp8":
        if not hasattr(torch, "float8_e4m3fn"):
            pytest.skip("torch without float8")
        a, b = a.to(torch.float8_e4m3fn), b.to(torch.float8_e4m3fn)
    slot = torch.zeros(8, dtype=torch.int64, device="cuda")
    ts = torch.zeros(4, dtype=torch.int64, device="cuda")
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    from dlnetbench_amd import _native
    hz = _native.lib().dlnb_wallclock_hz(0)  # the rate the ops convert with (measured against the host clock)
    for rep in range(3):
        ep = 1 + 3 * rep
        e0.record(s)
        gemm.gemm_deadline_ex(a, b, c, 2000.0, slot, ep, chain=False, tstart=(ts, 0), grid=_grid())
        gemm.idle_wait_us(300.0)  # a delay longer than a launch hop: absorbed only up to the cap
        gemm.gemm_deadline_ex(a, b, c, 3000.0, slot, ep + 1, chain=True, tstart=(ts, 1), grid=_grid())
        gemm.gemm_deadline_ex(a, b, c, 1000.0, slot, ep + 2, chain=True, tstart=(ts, 2), grid=_grid())
        e1.record(s)
        torch.cuda.synchronize()
    t = ts.tolist()
    # 2 ms + the 0.3 ms wait (+ its launch) - at most 30 us of it absorbed
    assert (2000 + 300 - 30) * 1e-6 * hz - 1 <= t[1] - t[0] <= (2000 + 300 + 60) * 1e-6 * hz, t
    assert abs(t[2] - t[1] - 3000e-6 * hz) <= 1, t  # a launch hop only: absorbed exactly
    ms = e0.elapsed_time(e1)
    # 2 + 3 + 1 ms + the unabsorbed part of the wait; the events bracket four launches (on a busy box the
    # first one's dispatch has added ~0.3 ms once in a full-suite run: the stamps above are the exact check)
    assert 6.27 <= ms <= 6.3 * 1.01 + 0.35, ms


def test_deadline_chain_counts_absorbed_lateness():
    """the lateness a chained task takes out of its own compute is counted, not only what
    exceeds the cap. Two chained deadline tasks back to back absorb the previous grid's drain and the launch
    hop; with a 10-us idle kernel between them ~10 us more (+ its launch); the second task still starts at the
    first's deadline and nothing is capped."""
    a, b, c = _deadline_operands()
    slot = torch.zeros(8, dtype=torch.int64, device="cuda")
    ts = torch.zeros(4, dtype=torch.int64, device="cuda")
    counters = torch.zeros(8, dtype=torch.int64, device="cuda")
    from dlnetbench_amd import _native
    hz = _native.lib().dlnb_wallclock_hz(0)
    absorbed = {}
    ep = 0
    for idle in (0.0, 10.0, 0.0, 10.0):  # each twice: the first round also loads the kernels
        counters.zero_()
        gemm.gemm_deadline_ex(a, b, c, 1000.0, slot, ep + 1, chain=False, tstart=(ts, 0), grid=_grid(),
                              counters=counters)
        if idle:
            gemm.idle_wait_us(idle)
        gemm.gemm_deadline_ex(a, b, c, 1000.0, slot, ep + 2, chain=True, tstart=(ts, 1), grid=_grid(),
                              counters=counters)
        torch.cuda.synchronize()
        ep += 2
        v = counters.tolist()
        t = ts.tolist()
        assert v[0] == 0 and v[1] == 0, v  # kCappedTasks, kCappedTicks: nothing beyond the 30-us cap
        assert v[5] == 1, v  # kAbsorbedTasks: the chained task came late and absorbed it
        assert abs(t[1] - t[0] - 1000e-6 * hz) <= 1, t  # it started at the first task's deadline
        absorbed[idle] = v[4] / hz * 1e6  # kAbsorbedTicks, us
    assert 0 < absorbed[0.0] < 25, absorbed
    assert 7 <= absorbed[10.0] - absorbed[0.0] <= 20, absorbed


def test_deadline_gate_waits_for_signal():
    """A gated task (deadline_sync.hpp) starts when its gate is raised on another stream (here after a
    4 ms idle wait there), not when its kernel launches, and a chained gated task whose gate opened after
    the previous deadline starts at the gate's time: the wait is exposed, never absorbed."""
    a, b, c = _deadline_operands()
    slot = torch.zeros(8, dtype=torch.int64, device="cuda")
    gates = torch.zeros(4, dtype=torch.int64, device="cuda")
    ts = torch.zeros(4, dtype=torch.int64, device="cuda")
    other = torch.cuda.Stream()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    mask = (1 << 48) - 1
    for rep in range(2):  # the first round also loads the kernels
        t0, t1 = 7 + 10 * rep, 9 + 10 * rep
        e0.record(s)
        other.wait_event(e0)
        # task 1: gate 0 raised right away; task 2 (chained): gate 1 raised ~4 ms after task 1's deadline
        with torch.cuda.stream(other):
            gemm.gate_signal_(gates, 0, t0)
            gemm.idle_wait_us(1000.0 + 4000.0)
            gemm.gate_signal_(gates, 1, t1)
        gemm.gemm_deadline_ex(a, b, c, 1000.0, slot, 1 + 2 * rep, chain=False, gates=[(gates, 0, t0)],
                              tstart=(ts, 0), grid=_grid())
        gemm.gemm_deadline_ex(a, b, c, 1000.0, slot, 2 + 2 * rep, chain=True, gates=[(gates, 1, t1), (gates, 0, t0)],
                              tstart=(ts, 1), grid=_grid())
        e1.record(s)
        torch.cuda.synchronize()
    g = gates.tolist()  # gate i = words [2i, 2i+1] = {seq, time}; seq = tag at iteration 0
    t = ts.tolist()
    assert g[0] == 17 and g[2] == 19, g
    gate1 = g[3] & mask
    assert (t[1] & mask) == gate1, (t, g)  # started at the late gate, not at the previous deadline
    from dlnetbench_amd import _native
    assert t[1] - t[0] >= round(4000e-6 * _native.lib().dlnb_wallclock_hz(0)) - 1, t
    ms = e0.elapsed_time(e1)
    assert 6.0 <= ms <= 6.0 * 1.02 + 0.1, ms
