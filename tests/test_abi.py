"""C-ABI boundary checks that need no GPU: the in-tree libtsdbhip.so loads,
exports every function include/tsdbhip.h declares, the ctypes structs match
the header layout, and opening a device without a GPU fails loudly."""
import ctypes as C
import os
import re

import pytest

from opentsdb_amd import _abi, _lib

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "tsdbhip.h")


def declared_functions():
    src = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|void|const char\*)\s+(tsdbhip_\w+)\s*\(", src, re.M)))


def test_header_declares_expected_entry_points():
    fns = declared_functions()
    assert set(_lib.EXPORTS) == set(fns), fns


def test_library_exports_every_declared_symbol():
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert L.tsdbhip_abi_version() == _abi.ABI_VERSION


def test_struct_sizes():
    # offsets/sizes fixed by the header (LP64)
    assert C.sizeof(_abi.SgDesc) == 8 + 8 + 4 + 4 + 4 + 4 + 8 + 6 * 8 + 8 + 8 + 8 + 8
    assert C.sizeof(_abi.SgOut) == 8 * 6 + 4 + 4 + 8
    assert C.sizeof(_abi.SynthParams) == 8 + 6 * 4


def test_open_without_gpu_fails_loudly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.TsdbHipError) as e:
        _lib.Context(0)
    assert e.value.code == _abi.E_NO_DEVICE
