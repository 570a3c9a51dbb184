import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session")
def engine():
    """One engine on cuda:0 for the whole GPU session (no fallback: fails loudly)."""
    from jobset_amd.engine import Engine
    e = Engine(0)
    yield e
    e.close()
