import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible MI355X (HIP) device")


@pytest.fixture(scope="session")
def coder():
    """The product HaarCoder; on a GPU run it must load the HIP library."""
    from wicca_amd import HaarCoder, _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible to libwicca_hip.so")
    return HaarCoder()
