import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP engine)")
    config.addinivalue_line("markers", "slow: large sizes (256 MiB class)")


@pytest.fixture(scope="session")
def gpu():
    """Fail loudly (not skip) when a gpu-marked test runs without the HIP engine."""
    import walrus_amd
    if not walrus_amd.device_available():
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    return walrus_amd
