import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); the parity tests proper")
    config.addinivalue_line("markers", "slow: longer CPU statistical checks")


@pytest.fixture(scope="session")
def kats():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def lib_path():
    """Path of the in-tree HIP engine library, built for gfx950 if stale (no GPU needed)."""
    from rsmcrt_amd import build as B
    return B.build()


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """torch ships its own HIP runtime next to /opt/rocm's, which libsmcrt.so uses. Whichever
    initialises the device second still works only if torch's came first (as in bench.py),
    so a GPU session initialises torch before any engine call."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass
    yield
