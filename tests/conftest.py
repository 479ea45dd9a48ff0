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


def pytest_terminal_summary(terminalreporter):
    """late call-end stamps (tsdbhip_timing.late_stamp: the snapshot's stamp
    seen only after spinning past the stream sync, the precursor of a stale
    read) over every context the session closed"""
    from opentsdb_amd import _lib
    s = _lib.STAMP_TOTALS
    if s["calls"]:
        terminalreporter.write_line(f"tsdbhip late_stamp: {s['late_stamp']} of {s['calls']} calls")
