import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "gnn-bfs-rans_amd")
for p in (REPO, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and libmignn.so")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(autouse=True)
def _no_device_errors(request):
    """After every GPU test: no launch may have recorded an in-kernel protocol
    failure (mignn_device_errors: e.g. a bounded LDS hand-off wait that ran
    out) -- such a launch's output is wrong even when the test's tolerance
    happened to hold."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import torch
    if not torch.cuda.is_available():
        return
    from mignn import _lib
    _lib.check_device_errors(request.node.name)
