"""Torch-facing wrappers for the hand-written CDNA4 kernels.

These call straight into libdlnb.so on torch's current HIP stream; there is
no fallback: on a GPU box a missing library is an error, never a silent
PyTorch path.
"""
from __future__ import annotations

from .. import _native


def _stream(t):
    import torch
    return torch.cuda.current_stream(t.device).cuda_stream


def gemm_tn(a, b, out=None, waves: int = 0):
    """C[M,N] (bf16) = A[M,K] @ B[N,K]^T with the 256x256 MFMA kernel.

    a, b: bf16 or float8_e4m3fn (OCP) CUDA tensors, row-major with K contiguous;
    rows may be strided (a view of a wider matrix: leading dimension = stride(0)).
    M and N must be multiples of 256; K*elem_size a multiple of 128 bytes;
    rows 16-byte aligned. out (optional) may be row-strided the same way.
    waves: the kernel variant (csrc/include/dlnb/kernels.hpp): 0 the default,
    5 one wave per SIMD MX (fp8), 6 8-phase, 8 8-wave double-buffered.
    """
    import torch
    if a.dtype != b.dtype:
        raise TypeError("a and b must have the same dtype")
    if a.dtype == torch.bfloat16:
        dt = _native.DTYPES["bf16"]
    elif a.dtype == getattr(torch, "float8_e4m3fn", None):
        dt = _native.DTYPES["fp8_e4m3"]
    else:
        raise TypeError(f"unsupported dtype {a.dtype}")
    M, K = a.shape
    N, K2 = b.shape
    if K != K2:
        raise ValueError("K mismatch")
    if a.stride(1) != 1 or b.stride(1) != 1:
        raise ValueError("a and b must be K-contiguous (row-major)")
    L = _native.lib()
    if not L.dlnb_gemm_shape_ok(M, N, K, dt):
        raise ValueError(f"unsupported shape M={M} N={N} K={K} (M,N % 256, K bytes % 128)")
    if out is None:
        out = torch.empty((M, N), device=a.device, dtype=torch.bfloat16)
    if out.stride(1) != 1:
        raise ValueError("out must be row-major")
    lda, ldb, ldc = a.stride(0), b.stride(0), out.stride(0)
    _native.check(L.dlnb_gemm_tn_waves(a.data_ptr(), b.data_ptr(), out.data_ptr(), M, N, K, lda, ldb, ldc, dt, waves,
                                       _stream(a)))
    return out


def gemm_deadline_us(a, b, c, us: float, stamp=None, grid: int = 0):
    """Persistent MFMA GEMM over C = A.B^T tiles that stops after `us` microseconds
    (device clock). `stamp` is a CUDA int64 tensor with >= 8 elements (the
    64-byte slot line the blocks agree their start through)."""
    import torch
    dt = _native.DTYPES["bf16"] if a.dtype == torch.bfloat16 else _native.DTYPES["fp8_e4m3"]
    M, K = a.shape
    N = b.shape[0]
    if stamp is None:
        stamp = torch.zeros(8, dtype=torch.int64, device=a.device)
    if stamp.numel() < 8 or stamp.dtype != torch.int64:
        # the kernels use words 0-2 of the 64-byte slot line (deadline_sync.hpp)
        raise ValueError("stamp must be an int64 tensor of >= 8 elements")
    _native.check(_native.lib().dlnb_gemm_deadline_us(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, dt, us,
                                                      a.device.index or 0, stamp.data_ptr(), grid, _stream(a)))
    return c


def gemm_deadline_ex(a, b, c, us: float, slot, epoch: int, chain=False, gates=(), tstart=None,
                     grid: int = 0, counters=None):
    """gemm_deadline_us with the whole start protocol (csrc/kernels/deadline_sync.hpp): `slot` an int64
    CUDA tensor of 8 elements reused by consecutive tasks of one stream, `epoch` the task number on it
    (1..65535, different from the previous task's), `chain` start at the slot's previous deadline
    absorbing at most `chain` us of lateness (True: the runtime's 30 us, DLNB_CHAIN_ABSORB_US),
    `gates` up to two (int64 CUDA tensor, gate index, tag) to wait for - gate i is the two words
    [2i, 2i+1] = {seq, time} (gate_signal_), `tstart` an (int64 tensor, index) that receives the
    task's start (s_memrealtime ticks), `counters` an int64 CUDA tensor of >= 8 elements the task adds
    its kernels::DlCounter counts to (capped / absorbed lateness, gate timeouts)."""
    import torch
    dt = _native.DTYPES["bf16"] if a.dtype == torch.bfloat16 else _native.DTYPES["fp8_e4m3"]
    M, K = a.shape
    N = b.shape[0]
    if slot.numel() < 8 or slot.dtype != torch.int64:
        raise ValueError("slot must be an int64 tensor of >= 8 elements")
    g = [(t.data_ptr() + 16 * i, tag) for t, i, tag in gates] + [(None, 0)] * (2 - len(gates))
    ts = tstart[0].data_ptr() + 8 * tstart[1] if tstart is not None else None
    if counters is not None and (counters.numel() < 8 or counters.dtype != torch.int64):
        raise ValueError("counters must be an int64 tensor of >= 8 elements")
    cp = counters.data_ptr() if counters is not None else None
    _native.check(_native.lib().dlnb_gemm_deadline_ex(a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, dt, us,
                                                      a.device.index or 0, slot.data_ptr(), grid, _stream(a), epoch,
                                                      30.0 if chain is True else float(chain or 0), g[0][0],
                                                      g[0][1], g[1][0], g[1][1], ts, cp))
    return c


def gate_signal_(gate, index: int, tag: int):
    """Raise gate `index` of an int64 CUDA tensor (words [2 index, 2 index + 1] = {seq = tag, time =
    s_memrealtime}) when torch's current stream reaches this point."""
    import torch
    if gate.numel() < 2 * index + 2 or gate.dtype != torch.int64:
        raise ValueError("gate must be an int64 tensor with two words per gate")
    _native.check(_native.lib().dlnb_gate_signal(gate.data_ptr() + 16 * index, tag, _stream(gate)))
    return gate


def fill_random_(t, seed: int = 0):
    """In-place uniform [-1, 1) fill with the native hash kernel."""
    import torch
    m = {torch.bfloat16: "bf16", torch.float16: "fp16", torch.float32: "fp32"}
    f8 = getattr(torch, "float8_e4m3fn", None)
    if f8 is not None:
        m[f8] = "fp8_e4m3"
    f85 = getattr(torch, "float8_e5m2", None)
    if f85 is not None:
        m[f85] = "fp8_e5m2"
    dt = _native.DTYPES[m[t.dtype]]
    _native.check(_native.lib().dlnb_fill_random(t.data_ptr(), t.numel(), dt, seed, _stream(t)))
    return t


def sgd_momentum_(param, mom, grad, lr: float = 1e-4, beta: float = 0.9):
    """param -= lr * (mom = beta*mom + grad), bf16 tensors, fp32 math."""
    _native.check(_native.lib().dlnb_sgd_momentum_bf16(param.data_ptr(), mom.data_ptr(), grad.data_ptr(),
                                                       param.numel(), lr, beta, _stream(param)))
    return param


def idle_wait_us(us: float, device: int = 0):
    import torch
    _native.check(_native.lib().dlnb_idle_wait_us(us, device, torch.cuda.current_stream(device).cuda_stream))


def busy_spin_us(us: float, device: int = 0):
    import torch
    _native.check(_native.lib().dlnb_busy_spin_us(us, device, torch.cuda.current_stream(device).cuda_stream))


def stamp_(slot, index: int = 0):
    """Write the device wall clock (s_memrealtime, 100 MHz) into slot[index] (int64 CUDA tensor)
    when torch's current stream reaches this point."""
    _native.check(_native.lib().dlnb_stamp(slot.data_ptr() + 8 * index, _stream(slot)))
    return slot


def gate_signal_iter_(gate, index: int, tag: int, iter_word):
    """gate_signal_ with the sequence (iteration << 32 | tag) read from iter_word[0] (int64 CUDA
    tensor) when the kernel runs."""
    _native.check(_native.lib().dlnb_gate_signal_iter(gate.data_ptr() + 16 * index, iter_word.data_ptr(), tag,
                                                      _stream(gate)))
    return gate


def task_size() -> int:
    """Bytes of one kernels::DlTask (a program's task list entry)."""
    return int(_native.lib().dlnb_task_size())


def program_ktiles(M: int, N: int, K: int, dtype) -> int:
    """K-tiles (128 bytes of K) of one tile of the program kernel for this shape (0: no program kernel)."""
    import torch
    dt = _native.DTYPES["bf16"] if dtype == torch.bfloat16 else _native.DTYPES["fp8_e4m3"]
    return int(_native.lib().dlnb_program_ktiles(M, N, K, dt))


def ptr(t, index: int = 0, words: int = 1) -> int:
    """Device address of word `index` (of `words` 8-byte words) of an int64 tensor / HostWords."""
    if isinstance(t, HostWords):
        return t.dev + 8 * index
    return t.data_ptr() + 8 * index


class HostWords:
    """n host-mapped, device-visible 64-bit words (hipHostMalloc mapped + coherent): `dev` is the
    device address, indexing reads / writes them from the host (e.g. an abort word)."""

    def __init__(self, n: int):
        import ctypes
        dev = ctypes.c_void_p()
        self.host = _native.lib().dlnb_host_words(n, ctypes.byref(dev))
        if not self.host:
            raise _native.NativeError("hipHostMalloc failed")
        self.dev = dev.value
        self.n = n
        self._arr = (ctypes.c_uint64 * n).from_address(self.host)

    def __getitem__(self, i: int) -> int:
        return int(self._arr[i])

    def __setitem__(self, i: int, v: int) -> None:
        self._arr[i] = v

    def free(self) -> None:
        if self.host:
            _native.lib().dlnb_host_words_free(self.host)
            self.host = None


def gemm_program(a, b, c, tasks, slot, task_buf, iter_word=None, counters=None, abort=None,
                 gate_timeout_s: float = 60.0, grid: int = 0, epoch: int = 0):
    """A compute program (kernels::gemm_tn_deadline_program): `tasks` a list of _native.TaskDesc
    (pointers as device addresses: see ptr()), `slot` an int64 CUDA tensor of 8 words (the stream's
    slot line), `task_buf` a uint8 / int64 CUDA tensor of >= len(tasks) * task_size() bytes the list
    is copied into (after torch's current stream is idle), `iter_word` an int64 CUDA tensor (the
    iteration word the gates' sequences and program claims read), `counters` an int64 CUDA tensor of
    >= 8 DlCounter words, `abort` a HostWords (word 0 the abort word). epoch 0: program claims from
    the iteration word; else a one-task launch epoch (1..65535)."""
    import torch
    dt = _native.DTYPES["bf16"] if a.dtype == torch.bfloat16 else _native.DTYPES["fp8_e4m3"]
    M, K = a.shape
    N = b.shape[0]
    if slot.numel() < 8 or slot.dtype != torch.int64:
        raise ValueError("slot must be an int64 tensor of >= 8 elements")
    if task_buf.numel() * task_buf.element_size() < len(tasks) * task_size():
        raise ValueError("task_buf too small")
    arr = (_native.TaskDesc * len(tasks))(*tasks)
    _native.check(_native.lib().dlnb_gemm_program(
        a.data_ptr(), b.data_ptr(), c.data_ptr(), M, N, K, dt, arr, len(tasks),
        iter_word.data_ptr() if iter_word is not None else None,
        counters.data_ptr() if counters is not None else None,
        abort.dev if abort is not None else None, gate_timeout_s, a.device.index or 0, slot.data_ptr(),
        task_buf.data_ptr(), grid, _stream(a), epoch))
    return c
