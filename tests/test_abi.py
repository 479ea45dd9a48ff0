"""C-ABI boundary checks: the in-tree libtsdbhip.so loads, exports every
function include/tsdbhip.h declares, the ctypes structs match the header
layout as a C compiler sees it (tests/abi_check.c, compiled against the
header and linked to the library: every struct's sizeof / offsetof against
_abi.py), and opening a device without a GPU fails loudly. On the GPU the
same C program runs a SpanGroup and a compaction through the .so."""
import ctypes as C
import json
import os
import re
import subprocess

import pytest

from opentsdb_amd import _abi, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tsdbhip.h")
CHECKER = os.path.join(ROOT, "tests", "_build", "abi_check")


def build_checker():
    """gcc, C11, -Werror: the header as a plain C consumer (the JNI shim) sees it."""
    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    os.makedirs(os.path.dirname(CHECKER), exist_ok=True)
    libdir = os.path.dirname(_lib.LIB_PATH)
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-O1", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "abi_check.c"), "-o", CHECKER, "-L", libdir, "-ltsdbhip",
                    f"-Wl,-rpath,{libdir}"], check=True)
    return CHECKER


CTYPES = {"tsdbhip_sg_desc": _abi.SgDesc, "tsdbhip_sg_out": _abi.SgOut, "tsdbhip_timing": _abi.Timing,
          "tsdbhip_rows_desc": _abi.RowsDesc, "tsdbhip_rows_out": _abi.RowsOut,
          "tsdbhip_synth_params": _abi.SynthParams}


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
    assert C.sizeof(_abi.SgDesc) == 8 + 8 + 4 + 4 + 4 + 4 + 8 + 6 * 8 + 8 + 8 + 8 + 8 + 8
    assert C.sizeof(_abi.SgOut) == 8 * 6 + 4 + 4 + 8
    assert C.sizeof(_abi.SynthParams) == 8 + 6 * 4


def test_c_layout_matches_ctypes():
    """sizeof / offsetof of every header struct, from C, == _abi.py's ctypes."""
    r = subprocess.run([build_checker(), "layout"], capture_output=True, text=True, check=True)
    d = json.loads(r.stdout)
    assert d["abi_version"] == _abi.ABI_VERSION
    assert set(d["structs"]) == set(CTYPES)
    for name, st in CTYPES.items():
        c = d["structs"][name]
        assert c["size"] == C.sizeof(st), name
        assert [f[0] for f in st._fields_] == list(c["fields"]), name
        for fname, ftype in st._fields_:
            off, size = c["fields"][fname]
            assert getattr(st, fname).offset == off, (name, fname)
            assert C.sizeof(ftype) == size, (name, fname)
    assert d["format"] == "sys.cpu 1356998400 42 host=a\nsys.cpu 1356998410 0.5 host=a\n"


@pytest.mark.gpu
def test_c_consumer_runs_on_gpu():
    """The C program drives a SpanGroup (KA-1) and a compaction through the .so."""
    r = subprocess.run([build_checker(), "run"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "bit-exact" in r.stdout


def test_open_without_gpu_fails_loudly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(_lib.TsdbHipError) as e:
        _lib.Context(0)
    assert e.value.code == _abi.E_NO_DEVICE
