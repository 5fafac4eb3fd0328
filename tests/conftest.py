import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests through the C-ABI")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def orbfe_lib():
    from orb_slam3_ros_amd import build
    build.build_library()
    from orb_slam3_ros_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu(orbfe_lib):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test but no HIP device is visible")
    torch.cuda.init()
    return torch.device("cuda:0")
