import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

DATA = os.path.join(ROOT, "data")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the HIP backend")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def native():
    from xflow_amd import native as nat

    return nat.load()


@pytest.fixture(scope="session")
def gpu_device():
    import torch

    from xflow_amd import native as nat

    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but torch sees no GPU")
    nat.require_hip()
    return torch.device("cuda", 0)
