import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build libmpx and the CLIs once per session (in-tree, incremental)."""
    jobs = str(min(8, os.cpu_count() or 1))
    res = subprocess.run(["make", "-C", ROOT, "-j", jobs, "all"], capture_output=True, text=True)
    if res.returncode != 0:
        pytest.exit(f"native build failed:\n{res.stdout[-4000:]}\n{res.stderr[-4000:]}", returncode=2)
    yield


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


@pytest.fixture
def root():
    return ROOT
