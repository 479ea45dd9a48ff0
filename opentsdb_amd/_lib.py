"""Loader for libtsdbhip.so (built in-tree by opentsdb_amd/csrc/Makefile).

There is no fallback: if the library or a GPU is missing, the product path
raises. `import torch` comes first so that the HIP runtime torch ships with
is the one libtsdbhip binds to (both use soname libamdhip64.so.7; loading
ours first would pull a second copy of the runtime into the process).
"""
import ctypes as C
import os
import subprocess

from . import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TSDBHIP_LIB") or os.path.join(HERE, "libtsdbhip.so")  # (override: A/B builds)
CSRC = os.path.join(HERE, "csrc")

_LIB = None

EXPORTS = [
    "tsdbhip_open", "tsdbhip_close", "tsdbhip_last_error", "tsdbhip_abi_version",
    "tsdbhip_host_register", "tsdbhip_host_unregister", "tsdbhip_spangroup_run",
    "tsdbhip_last_timing", "tsdbhip_compact_rows", "tsdbhip_comm_unique_id",
    "tsdbhip_comm_init", "tsdbhip_synth_generate", "tsdbhip_synth_free",
    "tsdbhip_desc_download", "tsdbhip_bw_probe", "tsdbhip_spangroup_run_batch",
    "tsdbhip_format_points", "tsdbhip_open_devices", "tsdbhip_open_mask", "tsdbhip_ranks",
    "tsdbhip_timing_totals", "tsdbhip_set_option",
]


class TsdbHipError(RuntimeError):
    def __init__(self, code, msg=""):
        self.code = code
        super().__init__(f"{_abi.ERR_NAMES.get(code, code)}: {msg}")


def build(force=False):
    """Compile libtsdbhip.so for gfx950 (hipcc cross-compiles without a GPU)."""
    args = ["make", "-s", "-C", CSRC]
    if force:
        args.append("-B")
    subprocess.run(args, check=True)


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    if not os.path.exists(LIB_PATH):
        raise TsdbHipError(_abi.E_NO_DEVICE, f"{LIB_PATH} not built; run opentsdb_amd._lib.build()")
    try:
        import torch  # noqa: F401  (pins the HIP runtime, see module doc)
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    L.tsdbhip_open.argtypes = [C.c_int32, P(C.c_void_p)]
    L.tsdbhip_open.restype = C.c_int
    L.tsdbhip_open_devices.argtypes = [P(C.c_int32), C.c_uint32, P(C.c_void_p)]
    L.tsdbhip_open_devices.restype = C.c_int
    L.tsdbhip_open_mask.argtypes = [C.c_uint32, P(C.c_void_p)]
    L.tsdbhip_open_mask.restype = C.c_int
    L.tsdbhip_set_option.argtypes = [C.c_void_p, C.c_char_p, C.c_char_p]
    L.tsdbhip_set_option.restype = C.c_int
    L.tsdbhip_ranks.argtypes = [C.c_void_p]
    L.tsdbhip_ranks.restype = C.c_int
    L.tsdbhip_close.argtypes = [C.c_void_p]
    L.tsdbhip_close.restype = None
    L.tsdbhip_last_error.argtypes = [C.c_void_p]
    L.tsdbhip_last_error.restype = C.c_char_p
    L.tsdbhip_abi_version.restype = C.c_int
    L.tsdbhip_host_register.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    L.tsdbhip_host_unregister.argtypes = [C.c_void_p, C.c_void_p]
    L.tsdbhip_spangroup_run.argtypes = [C.c_void_p, P(_abi.SgDesc), P(_abi.SgOut)]
    L.tsdbhip_spangroup_run.restype = C.c_int
    L.tsdbhip_spangroup_run_batch.argtypes = [C.c_void_p, P(_abi.SgDesc), C.c_uint32, P(C.c_uint32),
                                              P(_abi.SgOut)]
    L.tsdbhip_spangroup_run_batch.restype = C.c_int
    L.tsdbhip_format_points.argtypes = [C.c_int32, C.c_char_p, C.c_char_p, C.c_int64, P(C.c_int64),
                                        P(C.c_uint8), P(C.c_int64), C.c_uint64, C.c_char_p, C.c_uint64]
    L.tsdbhip_format_points.restype = C.c_int64
    L.tsdbhip_last_timing.argtypes = [C.c_void_p, P(_abi.Timing)]
    L.tsdbhip_timing_totals.argtypes = [C.c_void_p, P(_abi.Timing), P(C.c_uint64), C.c_int32]
    L.tsdbhip_compact_rows.argtypes = [C.c_void_p, P(_abi.RowsDesc), P(_abi.RowsOut)]
    L.tsdbhip_compact_rows.restype = C.c_int
    L.tsdbhip_comm_unique_id.argtypes = [C.c_char_p]
    L.tsdbhip_comm_init.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_char_p]
    L.tsdbhip_synth_generate.argtypes = [C.c_void_p, P(_abi.SynthParams), P(_abi.SgDesc)]
    L.tsdbhip_synth_free.argtypes = [C.c_void_p, P(_abi.SgDesc)]
    L.tsdbhip_desc_download.argtypes = [C.c_void_p, P(_abi.SgDesc)] + [C.c_void_p] * 8
    L.tsdbhip_bw_probe.argtypes = [C.c_void_p, P(_abi.SgDesc), C.c_int32, C.c_uint32, P(C.c_float),
                                   P(C.c_uint64)]
    L.tsdbhip_bw_probe.restype = C.c_int
    if L.tsdbhip_abi_version() != _abi.ABI_VERSION:
        raise TsdbHipError(_abi.E_INVALID_ARG, "ABI version mismatch")
    _LIB = L
    return L


# late call-end stamps (tsdbhip_timing.late_stamp) over every context closed
# in this process, and the calls they came from: the test suite's summary
# reports them (tests/conftest.py)
STAMP_TOTALS = {"late_stamp": 0, "calls": 0}


class Context:
    """One tsdbhip_ctx: a GPU (or, with `devices`, one shard per listed GPU of
    this process, a device may repeat), its pool of per-call streams and HBM
    scratch."""

    def __init__(self, device=0, devices=None):
        self._lib = lib()
        self._h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int32 * len(devices))(*[int(d) for d in devices])
            rc = self._lib.tsdbhip_open_devices(arr, len(devices), C.byref(self._h))
            device = int(devices[0])
        else:
            rc = self._lib.tsdbhip_open(int(device), C.byref(self._h))
        if rc:
            raise TsdbHipError(rc, self._lib.tsdbhip_last_error(None).decode())
        self.device = device
        self.ranks = self._lib.tsdbhip_ranks(self._h)

    @property
    def handle(self):
        return self._h

    def last_error(self):
        return self._lib.tsdbhip_last_error(self._h).decode()

    def check(self, rc):
        if rc:
            raise TsdbHipError(rc, self.last_error())

    def set_option(self, name, value):
        """tsdbhip_set_option: a path / diagnostic option of this context
        (include/tsdbhip.h); results never depend on it"""
        self.check(self._lib.tsdbhip_set_option(self._h, name.encode(), value.encode()))

    def timing(self):
        t = _abi.Timing()
        self._lib.tsdbhip_last_timing(self._h, C.byref(t))
        return t

    def timing_totals(self, reset=False):
        """(sums of the timing fields over the calls since the last reset, number of calls)"""
        t, n = _abi.Timing(), C.c_uint64()
        self._lib.tsdbhip_timing_totals(self._h, C.byref(t), C.byref(n), 1 if reset else 0)
        return t, int(n.value)

    def comm_init(self, nranks, rank, uid):
        self.check(self._lib.tsdbhip_comm_init(self._h, nranks, rank, uid))

    @staticmethod
    def unique_id():
        buf = C.create_string_buffer(_abi.UNIQUE_ID_BYTES)
        rc = lib().tsdbhip_comm_unique_id(buf)
        if rc:
            raise TsdbHipError(rc, lib().tsdbhip_last_error(None).decode())
        return buf.raw

    def close(self):
        if self._h:
            try:
                t, n = self.timing_totals()
                STAMP_TOTALS["late_stamp"] += int(t.late_stamp)
                STAMP_TOTALS["calls"] += n
            except Exception:  # (bookkeeping only)
                pass
            self._lib.tsdbhip_close(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
