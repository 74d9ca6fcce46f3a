import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm MI355X device (run on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    import numpy as np

    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = dict(np.load(GOLDEN / f"{name}.npz", allow_pickle=False))
        return cache[name]

    return load


@pytest.fixture(autouse=True)
def _torch_seed(request):
    """torch's global generator seeded per test from its node id: tests that draw with
    torch.randn get the same inputs whichever tests ran before them (a test's float64
    comparison must not depend on the suite's order or selection)."""
    import zlib
    try:
        import torch
    except Exception:
        return
    torch.manual_seed(zlib.crc32(request.node.nodeid.encode()))


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no ROCm device is visible")
    from graphneuralnetwork_amd import _lib
    _lib.load()  # fail loudly if the HIP library is missing
    return torch.device("cuda:0")
