"""ctypes binding to the native runtime (dlnetbench_amd/_lib/libdlnb.so).

The library is built in-tree (``make`` or ``__graft_entry__.build()``) so it
travels with the repository. torch (when installed) is imported *first*: its
wheel bundles libamdhip64.so / librccl.so with the same sonames as
/opt/rocm, and loading torch first makes the dynamic loader resolve our
library's HIP/RCCL dependencies to the already-loaded copies, so one process
never ends up with two HIP runtimes. DLNB_NO_TORCH=1 skips that import (the
process then runs entirely on /opt/rocm's HIP and RCCL, like the CLI binaries;
do not import torch afterwards in such a process).
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import List, Optional

_LIB: Optional[ctypes.CDLL] = None
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libdlnb.so")

# dlnb::DType values (csrc/include/dlnb/common.hpp)
DTYPES = {"bf16": 0, "fp16": 1, "fp32": 2, "fp8": 3, "fp8_e4m3": 3, "fp8_e5m2": 4}


class NativeError(RuntimeError):
    pass


class TaskDesc(ctypes.Structure):
    """One task of a compute program (csrc/src/capi.cpp dlnb_task_desc ->
    kernels::DlTask): ticks > 0 a deadline task, ticks == 0 with work_rounds /
    tail_kt a fixed-work task, flags = 1 a gate-only task (its gates, then its
    done gate), none of these the join."""
    _fields_ = [("ticks", ctypes.c_ulonglong), ("chain_ticks", ctypes.c_ulonglong),
                ("gate0", ctypes.c_void_p), ("gate1", ctypes.c_void_p),
                ("tag0", ctypes.c_uint), ("tag1", ctypes.c_uint),
                ("tstart0", ctypes.c_void_p), ("tstart1", ctypes.c_void_p),
                ("done_gate", ctypes.c_void_p), ("done_tag", ctypes.c_uint),
                ("work_rounds", ctypes.c_uint), ("tail_kt", ctypes.c_uint), ("epoch", ctypes.c_uint),
                ("tend", ctypes.c_void_p), ("flags", ctypes.c_uint)]


def lib() -> ctypes.CDLL:
    global _LIB
    if _LIB is not None:
        return _LIB
    if os.environ.get("DLNB_NO_TORCH", "0") != "1":
        try:  # see module docstring
            import torch  # noqa: F401
        except ImportError:
            pass
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} is missing: build it with `make` (or __graft_entry__.build())")
    # RTLD_LOCAL: with RTLD_GLOBAL, the library's (and its HIP / RCCL
    # dependencies') exported symbols interposed on extension modules dlopen'ed
    # later in the process - the hypothesis pytest plugin's native module
    # segfaulted on import at the end of a full test session (exit 139)
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_LOCAL)
    c_int, c_size, c_vp, c_dbl, c_float = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_double, ctypes.c_float
    L.dlnb_version.restype = ctypes.c_char_p
    L.dlnb_last_error.restype = ctypes.c_char_p
    L.dlnb_free.argtypes = [c_vp]
    L.dlnb_gpu_count.restype = c_int
    L.dlnb_run.argtypes = [ctypes.c_char_p, c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(c_vp)]
    L.dlnb_run.restype = c_int
    L.dlnb_parse_stats.argtypes = [ctypes.c_char_p, ctypes.POINTER(c_vp)]
    L.dlnb_parse_stats.restype = c_int
    L.dlnb_fill_random.argtypes = [c_vp, c_size, c_int, ctypes.c_ulonglong, c_vp]
    L.dlnb_gemm_tn.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]
    L.dlnb_gemm_tn_waves.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_vp]
    L.dlnb_gemm_deadline_us.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_dbl, c_int, c_vp, c_int, c_vp]
    L.dlnb_gemm_deadline_ex.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, c_dbl, c_int, c_vp, c_int, c_vp,
                                        ctypes.c_uint, c_dbl, c_vp, ctypes.c_uint, c_vp, ctypes.c_uint, c_vp, c_vp]
    L.dlnb_gate_signal.argtypes = [c_vp, ctypes.c_uint, c_vp]
    L.dlnb_gate_signal_iter.argtypes = [c_vp, c_vp, ctypes.c_uint, c_vp]
    L.dlnb_task_size.restype = c_int
    L.dlnb_gemm_program.argtypes = [c_vp, c_vp, c_vp, c_int, c_int, c_int, c_int, ctypes.POINTER(TaskDesc), c_int,
                                    c_vp, c_vp, c_vp, c_dbl, c_int, c_vp, c_vp, c_int, c_vp, ctypes.c_uint]
    L.dlnb_program_ktiles.argtypes = [c_int, c_int, c_int, c_int]
    L.dlnb_host_words.argtypes = [c_int, ctypes.POINTER(c_vp)]
    L.dlnb_host_words.restype = c_vp
    L.dlnb_host_words_free.argtypes = [c_vp]
    L.dlnb_gemm_shape_ok.argtypes = [c_int, c_int, c_int, c_int]
    L.dlnb_gemm_narrow_nf.argtypes = [c_int, c_int, c_int]
    L.dlnb_idle_wait_us.argtypes = [c_dbl, c_int, c_vp]
    L.dlnb_busy_spin_us.argtypes = [c_dbl, c_int, c_vp]
    L.dlnb_sgd_momentum_bf16.argtypes = [c_vp, c_vp, c_vp, c_size, c_float, c_float, c_vp]
    L.dlnb_stamp.argtypes = [c_vp, c_vp]
    L.dlnb_wallclock_hz.argtypes = [c_int]
    L.dlnb_wallclock_hz.restype = c_dbl
    L.dlnb_bf16_to_float.argtypes = [ctypes.c_ushort]
    L.dlnb_bf16_to_float.restype = c_float
    L.dlnb_float_to_bf16.argtypes = [c_float]
    L.dlnb_float_to_bf16.restype = ctypes.c_ushort
    L.dlnb_fp8e4m3_to_float.argtypes = [ctypes.c_ubyte]
    L.dlnb_fp8e4m3_to_float.restype = c_float
    L.dlnb_float_to_fp8e4m3.argtypes = [c_float]
    L.dlnb_float_to_fp8e4m3.restype = ctypes.c_ubyte
    _LIB = L
    return L


def check(rc: int) -> None:
    if rc != 0:
        raise NativeError(lib().dlnb_last_error().decode())


def _take_string(ptr: ctypes.c_void_p) -> str:
    s = ctypes.cast(ptr, ctypes.c_char_p).value.decode()
    lib().dlnb_free(ptr)
    return s


def version() -> str:
    return lib().dlnb_version().decode()


def run_raw(strategy: str, args: List[str]) -> dict:
    """Run a benchmark in-process; returns the report document."""
    L = lib()
    argv = (ctypes.c_char_p * len(args))(*[a.encode() for a in args])
    out = ctypes.c_void_p()
    check(L.dlnb_run(strategy.encode(), len(args), argv, ctypes.byref(out)))
    return json.loads(_take_string(out)) if out.value else {}


def parse_stats(path: str) -> dict:
    out = ctypes.c_void_p()
    check(lib().dlnb_parse_stats(path.encode(), ctypes.byref(out)))
    return json.loads(_take_string(out))
