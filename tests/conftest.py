import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: multi-process or long-running test")


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributedtensorflowexample_amd.ops import hip

    hip()  # loud failure if the kernels are missing on a GPU box
    return torch.device("cuda:0")


@pytest.fixture(scope="session")
def native_host():
    from distributedtensorflowexample_amd.ops import host

    return host()
