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
