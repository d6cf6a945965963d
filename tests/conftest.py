import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built xdot/_C.so")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import xdot._ext as ext

    assert ext.load(), "xdot/_C.so must be built and loadable on a GPU box"
    return torch.device("cuda", 0)
