import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through libhipquorum.so)")


@pytest.fixture(scope="session")
def hq():
    """The product binding; raises (never skips) when the HIP library is missing."""
    from dragonboat_amd import hipquorum

    return hipquorum


@pytest.fixture(scope="session")
def gpu_ctx(hq):
    ctx = hq.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def oracle():
    from oracle import qref

    return qref
