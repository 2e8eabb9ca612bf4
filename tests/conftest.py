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
    # (re)build when the library is missing or its embedded build id is not
    # this tree's (build.source_id); build_lib recompiles only stale objects
    if not os.path.exists(_lib.LIB_PATH) or _embedded_id(_lib.LIB_PATH) != build.source_id():
        build.build_lib()
    from tests.rccl_shim import build as shim  # the test-only RCCL stand-in (test_shim_ranks_gather)
    shim.build()
    yield


def _embedded_id(path):
    """rt_build_id() of a built library, read without loading it."""
    import re
    with open(path, "rb") as fp:
        m = re.search(rb"generated-id:([0-9a-f]{64})", fp.read())
    return m.group(1).decode() if m else None
