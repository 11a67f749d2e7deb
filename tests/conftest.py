import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "raytracing-book_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) — run with -m gpu")
    config.addinivalue_line("markers", "slow: longer CPU test")


def gpu_available():
    try:
        import rtamd
        return rtamd.amd().rt_debug_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Loads the HIP library; fails loudly (no fallback) when it cannot."""
    import rtamd
    L = rtamd.amd()
    n = L.rt_debug_device_count()
    assert n > 0, "no HIP device visible to a -m gpu test"
    return L
