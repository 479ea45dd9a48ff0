import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs libtsdbhip kernels)")


@pytest.fixture(scope="session")
def ctx():
    from opentsdb_amd._lib import Context
    c = Context(0)
    yield c
    c.close()
