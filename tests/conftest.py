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
    # An existing host-ASan build is brought up to date (incremental) so its
    # tests never run stale binaries.
    if os.path.isdir(os.path.join(ROOT, "build-asan", "bin")) and not os.environ.get("PYTEST_XDIST_WORKER"):
        subprocess.run(["make", "-C", ROOT, f"-j{min(16, os.cpu_count() or 4)}", "asan"], check=False,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
