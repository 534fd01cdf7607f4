import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device + native kernels)")
    config.addinivalue_line("markers", "slow: longer multi-process tests")


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from harp_amd.ops import _lib

    _lib.kernels()  # native library must load on a GPU box (fail loudly, no fallback)
    return torch.device("cuda", 0)
