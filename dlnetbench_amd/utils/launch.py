"""Process launcher: ``python -m dlnetbench_amd.utils.launch -n N <program> [args...]``.

The reference is launched with ``mpirun -n N`` / ``srun`` and bootstraps over
MPI. There is no MPI on the target image; this launcher
forks N ranks on one node with DLNB_RANK / DLNB_WORLD_SIZE /
DLNB_LOCAL_RANK / DLNB_LOCAL_WORLD_SIZE and DLNB_STORE_ADDR (the TCP
rendezvous store hosted by rank 0). The native runtime also understands
torchrun, Open MPI, PMI and Slurm variables, so ``torchrun --no-python`` or
``srun`` work as well. If one rank fails, the others are terminated.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def rank_env(rank: int, world: int, store_file: str, base: Optional[Dict[str, str]] = None) -> Dict[str, str]:
    env = dict(os.environ if base is None else base)
    env.pop("DLNB_STORE_ADDR", None)
    env.update({
        "DLNB_RANK": str(rank),
        "DLNB_WORLD_SIZE": str(world),
        "DLNB_LOCAL_RANK": str(rank),
        "DLNB_LOCAL_WORLD_SIZE": str(world),
        # rank 0 serves the store on an ephemeral port and publishes it here
        "DLNB_STORE_FILE": store_file,
        # dmabuf IPC only on this pool (RCCL / tensor sharing across processes)
        "HSA_ENABLE_IPC_MODE_LEGACY": env.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
    })
    # Do not let an outer torchrun/MPI identity leak into the children.
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "OMPI_COMM_WORLD_RANK",
              "OMPI_COMM_WORLD_SIZE", "PMI_RANK", "PMI_SIZE", "SLURM_PROCID", "SLURM_NTASKS"):
        env.pop(k, None)
    return env


def launch(n: int, cmd: Sequence[str], timeout: Optional[float] = None, capture: bool = False,
           env: Optional[Dict[str, str]] = None, cwd: Optional[str] = None):
    """Start n ranks of cmd; returns (exit_code, [stdout per rank] or None)."""
    import shutil
    import tempfile
    rdv = tempfile.mkdtemp(prefix="dlnb_rdv_")
    store_file = os.path.join(rdv, "store")
    procs: List[subprocess.Popen] = []
    outs: List[Optional[str]] = [None] * n
    for r in range(n):
        procs.append(subprocess.Popen(
            list(cmd), env=rank_env(r, n, store_file, env), cwd=cwd,
            stdout=subprocess.PIPE if capture else None,
            stderr=subprocess.STDOUT if capture else None,
            start_new_session=True, text=True))
    t0 = time.time()
    code = 0
    try:
        if capture:
            import threading

            def reader(i):
                outs[i] = procs[i].stdout.read()
            ths = [threading.Thread(target=reader, args=(i,), daemon=True) for i in range(n)]
            for t in ths:
                t.start()
        alive = set(range(n))
        while alive:
            for i in list(alive):
                rc = procs[i].poll()
                if rc is not None:
                    alive.discard(i)
                    if rc != 0 and code == 0:
                        code = rc
                        _kill_all(procs)
            if timeout is not None and time.time() - t0 > timeout:
                _kill_all(procs)
                code = code or 124
                break
            time.sleep(0.02)
        for p in procs:
            try:
                p.wait(timeout=10)
            except subprocess.TimeoutExpired:
                os.killpg(p.pid, signal.SIGKILL)
        if capture:
            for t in ths:
                t.join(timeout=10)
    except KeyboardInterrupt:
        _kill_all(procs)
        raise
    finally:
        shutil.rmtree(rdv, ignore_errors=True)
    return code, (outs if capture else None)


def _kill_all(procs: List[subprocess.Popen]) -> None:
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, signal.SIGTERM)
            except ProcessLookupError:
                pass


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("-n", "--nproc", type=int, required=True, help="number of ranks")
    ap.add_argument("--timeout", type=float, default=None, help="kill the job after this many seconds")
    ap.add_argument("cmd", nargs=argparse.REMAINDER)
    a = ap.parse_args(argv)
    cmd = a.cmd[1:] if a.cmd and a.cmd[0] == "--" else a.cmd
    if not cmd:
        ap.error("missing program")
    code, _ = launch(a.nproc, cmd, timeout=a.timeout)
    return code


if __name__ == "__main__":
    sys.exit(main())
