import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    # build the product library and the oracle once per session (no-ops when fresh)
    from lsm_amd import _build
    _build.build()
    from oracle import oracle
    oracle.build()
