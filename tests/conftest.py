import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (run with -m gpu on MI355X)")
    config.addinivalue_line("markers", "slow: full-size parity (BASELINE sizes)")


@pytest.fixture(scope="session")
def sva():
    import stereovisionarray_amd as m
    return m


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    return pyoracle


@pytest.fixture(scope="session")
def ctx(sva):
    """One context on cuda:0 that shares torch's current stream, so torch's
    allocations/fills and the sva kernels are stream-ordered."""
    if sva.device_count() < 1:
        pytest.fail("GPU test selected but no HIP device is visible")
    import torch
    c = sva.Context(0)
    s = torch.cuda.Stream(torch.device("cuda:0"))
    torch.cuda.set_stream(s)
    c.set_stream(s.cuda_stream)
    yield c
    c.close()


@pytest.fixture(scope="session")
def torch_dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but torch sees no device")
    return torch.device("cuda:0")
