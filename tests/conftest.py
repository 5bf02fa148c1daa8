import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblorb.so / HIP)")


@pytest.fixture(scope="session")
def ctx():
    """One lorb_ctx for the whole GPU session (one process, one stream)."""
    from lorb_slam_amd.runtime import Context
    c = Context(0)  # raises loudly if liblorb.so is missing or no device is visible
    yield c
    c.close()
