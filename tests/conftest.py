import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through librpgpu.so on the device)")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def rplib():
    """The product library (C-ABI).  Loading needs no GPU."""
    from redpanda_amd import build as B
    from redpanda_amd import _lib
    if not os.path.exists(_lib.LIB_PATH):
        B.build()
    return _lib


@pytest.fixture(scope="session")
def engine():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from redpanda_amd.engine import Engine
    return Engine(0)
