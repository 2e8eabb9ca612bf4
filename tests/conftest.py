import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long CPU test")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Build the oracle (gcc) and the HIP library (hipcc) if they are missing."""
    from oracle import _oracle
    if not os.path.exists(_oracle._LIB_PATH):
        _oracle.build()
    from cpp_cuda_raytracer_dev_amd import _lib, build
    if not os.path.exists(_lib.LIB_PATH):
        build.build_lib()
    yield
