import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP solver)")
    config.addinivalue_line("markers", "slow: large-size case")


@pytest.fixture(scope="session", autouse=True)
def _built():
    import __graft_entry__

    __graft_entry__.build()
    yield


@pytest.fixture(autouse=True)
def _default_precision():
    from oracle import pyoracle as O
    from simgrid_amd import lmm

    lmm.set_precision(1e-5)
    O.set_precision(1e-5)
    yield
    lmm.set_precision(1e-5)
    O.set_precision(1e-5)
