import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on a GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def root():
    return ROOT


@pytest.fixture(scope="session")
def data_dir():
    return os.path.join(ROOT, "tests", "data")


def pytest_sessionstart(session):
    """Build the native library and binaries if this checkout has not been built."""
    import subprocess
    need = [os.path.join(ROOT, "dlnetbench_amd", "_lib", "libdlnb.so"), os.path.join(ROOT, "build", "bin", "dp")]
    if not all(os.path.exists(p) for p in need) and not os.environ.get("PYTEST_XDIST_WORKER"):
        subprocess.run(["make", "-C", ROOT, f"-j{min(16, os.cpu_count() or 4)}"], check=True,
                       stdout=subprocess.DEVNULL)


def _sanitizer_build(kind: str) -> str:
    """`make asan` / `make tsan` into build-<kind>/ (incremental: the first
    session compiles the tree once, later ones only what changed) and return
    its bin directory. A failing build fails the tests that need it."""
    import fcntl
    import subprocess
    # one make per tree at a time: pytest-xdist workers each build the session fixture, and two makes
    # relinking build-<kind>/libdlnb.so under each other fail the link of the binaries
    with open(os.path.join(ROOT, f".build-{kind}.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        p = subprocess.run(["make", "-C", ROOT, f"-j{min(16, os.cpu_count() or 4)}", kind], capture_output=True,
                           text=True)
    assert p.returncode == 0, f"make {kind} failed:\n" + p.stdout[-2000:] + p.stderr[-3000:]
    return os.path.join(ROOT, f"build-{kind}", "bin")


@pytest.fixture(scope="session")
def asan_bindir():
    return _sanitizer_build("asan")


@pytest.fixture(scope="session")
def tsan_bindir():
    return _sanitizer_build("tsan")
