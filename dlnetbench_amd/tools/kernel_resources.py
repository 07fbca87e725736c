"""Per-kernel register / LDS / scratch usage of a HIP source, read from the
gfx950 code object (no GPU needed: hipcc cross-compiles here).

    python -m dlnetbench_amd.tools.kernel_resources csrc/kernels/xgmi.hip [--json]

For each kernel: VGPRs, AGPRs, SGPRs, LDS bytes, scratch bytes and the waves
per SIMD its registers allow (CDNA4: 512 registers per SIMD lane shared by
VGPRs + AGPRs in 8-register granules, at most 8 waves per SIMD), plus the
blocks of its declared size that fit one CU on registers alone. The xgmi
backend's CU budget (comm_xgmi.cpp) relies on 4 blocks of 512 threads per CU,
i.e. <= 64 registers per lane; tests/test_tools.py checks that here.
"""
from __future__ import annotations

import argparse
import json
import os
import re
import subprocess
import tempfile
from typing import Dict, List

ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _demangle(names: List[str]) -> List[str]:
    for tool in (os.path.join(ROCM, "lib/llvm/bin/llvm-cxxfilt"), "c++filt"):
        try:
            p = subprocess.run([tool], input="\n".join(names), capture_output=True, text=True, check=True)
            out = p.stdout.splitlines()
            if len(out) == len(names):
                return out
        except (OSError, subprocess.CalledProcessError):
            continue
    return names


def waves_per_simd(vgpr: int, agpr: int) -> int:
    regs = vgpr + agpr
    regs = (regs + 7) // 8 * 8 if regs else 8
    return max(0, min(8, 512 // regs))


def kernel_resources(src: str, arch: str = "gfx950", extra: List[str] = ()) -> List[Dict]:
    """Compile `src` for `arch` (device only) and return one dict per kernel."""
    with tempfile.TemporaryDirectory() as td:
        bundle = os.path.join(td, "k.o")
        co = os.path.join(td, "k.co")
        subprocess.run([os.path.join(ROCM, "bin/hipcc"), "-O3", "-std=c++17", f"-I{ROOT}/csrc/include",
                        f"--offload-arch={arch}", "--cuda-device-only", "-c", src, "-o", bundle, *extra],
                       check=True, capture_output=True, text=True)
        subprocess.run([os.path.join(ROCM, "lib/llvm/bin/clang-offload-bundler"), "--unbundle", "--type=o",
                        f"--input={bundle}", f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}", f"--output={co}"],
                       check=True, capture_output=True, text=True)
        notes = subprocess.run([os.path.join(ROCM, "lib/llvm/bin/llvm-readelf"), "--notes", co],
                               check=True, capture_output=True, text=True).stdout
    # The metadata is YAML-like: one "- .args/..." record per kernel; keys we
    # need are flat ".key: value" lines inside each record.
    kernels: List[Dict] = []
    cur: Dict = {}
    keys = {".name": "name", ".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
            ".group_segment_fixed_size": "lds", ".private_segment_fixed_size": "scratch",
            ".max_flat_workgroup_size": "max_threads"}
    for line in notes.splitlines():
        m = re.match(r"^\s*(?:- )?(\.[a-z_]+):\s+(\S+)\s*$", line)
        if not m or m.group(1) not in keys:
            continue
        k, v = keys[m.group(1)], m.group(2)
        if k == "name":
            cur["name"] = v
        else:
            cur[k] = int(v)
        if all(x in cur for x in ("name", "vgpr", "agpr", "sgpr", "lds", "scratch", "max_threads")):
            kernels.append(cur)
            cur = {}
    names = _demangle([k["name"] for k in kernels])
    for k, n in zip(kernels, names):
        k["symbol"] = k["name"]
        k["name"] = n
        w = waves_per_simd(k["vgpr"], k["agpr"])
        k["waves_per_simd"] = w
        waves_per_block = max(1, (k["max_threads"] + 63) // 64)
        # 4 SIMDs per CU; a block's waves spread over them
        k["blocks_per_cu_regs"] = (4 * w) // waves_per_block
    return kernels


def main() -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("sources", nargs="+")
    ap.add_argument("--arch", default="gfx950")
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    rows = []
    for s in a.sources:
        for k in kernel_resources(s, a.arch):
            k["source"] = os.path.relpath(s, ROOT)
            rows.append(k)
    if a.json:
        print(json.dumps(rows, indent=1))
        return 0
    print(f"{'vgpr':>5} {'agpr':>5} {'sgpr':>5} {'lds':>7} {'scratch':>7} {'waves/SIMD':>10} {'blk/CU':>6}  kernel")
    for k in rows:
        print(f"{k['vgpr']:>5} {k['agpr']:>5} {k['sgpr']:>5} {k['lds']:>7} {k['scratch']:>7} "
              f"{k['waves_per_simd']:>10} {k['blocks_per_cu_regs']:>6}  {k['name'][:110]}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
