import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "hybrid-vehicle-platoon_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    config.addinivalue_line("markers", "slow: longer CPU cross-checks")


@pytest.fixture(scope="session")
def gpu_available():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return True
