"""tsdbhip_host_register / _unregister across contexts: a
HIP registration is process-wide, so two contexts registering the same host
buffer share it, and only the last unregister releases it."""
import ctypes as C

import numpy as np
import pytest

from opentsdb_amd import _abi

pytestmark = pytest.mark.gpu


def test_shared_registration_is_reference_counted(ctx):
    from opentsdb_amd._lib import Context
    other = Context(0)
    try:
        buf = np.zeros(1 << 16, dtype=np.uint8)
        p = buf.ctypes.data_as(C.c_void_p)
        L = ctx._lib
        assert L.tsdbhip_host_register(ctx.handle, p, buf.nbytes) == _abi.OK
        assert L.tsdbhip_host_register(other.handle, p, buf.nbytes) == _abi.OK
        # (a different length for the same pointer is refused, the entry kept)
        assert L.tsdbhip_host_register(other.handle, p, buf.nbytes // 2) == _abi.E_INVALID_ARG
        assert L.tsdbhip_host_unregister(ctx.handle, p) == _abi.OK
        # still registered for `other`: its unregister releases the HIP registration
        assert L.tsdbhip_host_unregister(other.handle, p) == _abi.OK
        # nothing left to release
        assert L.tsdbhip_host_unregister(other.handle, p) != _abi.OK
    finally:
        other.close()
