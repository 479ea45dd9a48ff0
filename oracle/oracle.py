"""ctypes wrapper of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference path (see oracle.cc header). Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as
the checker or the timed CPU baseline; the product package never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from opentsdb_amd import _abi

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = C.CDLL(path)
        L.oracle_spangroup_run.argtypes = [C.POINTER(_abi.SgDesc), C.POINTER(_abi.SgOut)]
        L.oracle_spangroup_run.restype = C.c_int
        L.oracle_agg_long.argtypes = [C.c_int, C.POINTER(C.c_int64), C.c_size_t, C.POINTER(C.c_int64)]
        L.oracle_agg_double.argtypes = [C.c_int, C.POINTER(C.c_double), C.c_size_t, C.POINTER(C.c_double)]
        L.oracle_compact_rows.argtypes = [C.POINTER(_abi.RowsDesc), C.POINTER(_abi.RowsOut)]
        L.oracle_compact_rows.restype = C.c_int
        L.oracle_regular_sharded.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                             C.c_uint32, C.c_int64, C.c_int64, C.c_int, C.c_int, C.c_int32,
                                             C.c_int, C.c_uint32, C.c_int, C.POINTER(_abi.SgOut)]
        L.oracle_regular_sharded.restype = C.c_int
        _LIB = L
    return _LIB


class Result:
    def __init__(self, code, ts, is_int, bits, n_input, err_index):
        self.code = code
        self.ts = ts
        self.is_int = is_int
        self.bits = bits
        self.n_input_points = n_input
        self.err_index = err_index

    def values(self):
        """Python values: int for integer points, float otherwise."""
        d = self.bits.view(np.float64)
        return [int(self.bits[i]) if self.is_int[i] else float(d[i]) for i in range(len(self.ts))]

    def __repr__(self):
        return f"Result(code={self.code}, n={len(self.ts)}, n_input={self.n_input_points})"


def spangroup(spanset, start, end, agg, rate=False, ds_interval=0, ds_agg=0, capacity=None):
    desc = _abi.SgDesc()
    spanset.fill_desc(desc)
    desc.start_time, desc.end_time = int(start), int(end)
    desc.rate, desc.agg, desc.ds_agg = int(bool(rate)), int(agg), int(ds_agg)
    desc.ds_interval = int(ds_interval)
    desc.flags = 0
    cap = int(capacity if capacity is not None else max(1, spanset.n_cells()))
    ts = np.zeros(cap, np.int64)
    isi = np.zeros(cap, np.uint8)
    bits = np.zeros(cap, np.int64)
    out = _abi.SgOut()
    out.capacity = cap
    out.ts = _abi.ptr(ts, C.c_int64)
    out.is_int = _abi.ptr(isi, C.c_uint8)
    out.bits = _abi.ptr(bits, C.c_int64)
    code = lib().oracle_spangroup_run(C.byref(desc), C.byref(out))
    n = int(out.n_out)
    return Result(code, ts[:n].copy(), isi[:n].copy(), bits[:n].copy(),
                  int(out.n_input_points), int(out.err_index))


def regular_sharded(n_spans, n_points, kind, seed, step, start, end, agg, rate=False, ds_interval=0, ds_agg=0,
                    t0=None, shard_spans=2000, threads=None, capacity=None):
    """The synthetic regular SpanGroup of synth.regular / tsdbhip_synth_generate
    at full size, generated and iterated shard by shard on host threads and
    combined in shard order (oracle.cc: oracle_regular_sharded; sum / min /
    max on aligned grids only, and dev on the double path as a pairwise merge
    of the shards' Welford states)."""
    from opentsdb_amd import synth
    t0 = synth.T0 if t0 is None else t0
    cap = int(capacity or max(1, n_points if not ds_interval else n_points * step // ds_interval + 2))
    ts, isi, bits = np.zeros(cap, np.int64), np.zeros(cap, np.uint8), np.zeros(cap, np.int64)
    out = _abi.SgOut(capacity=cap, ts=_abi.ptr(ts, C.c_int64), is_int=_abi.ptr(isi, C.c_uint8),
                     bits=_abi.ptr(bits, C.c_int64))
    threads = threads or max(1, min(16, os.cpu_count() or 1))
    code = lib().oracle_regular_sharded(seed, n_spans, n_points, t0, step, kind, int(start), int(end), agg,
                                        int(bool(rate)), ds_interval, ds_agg, shard_spans, threads, C.byref(out))
    n = int(out.n_out)
    return Result(code, ts[:n].copy(), isi[:n].copy(), bits[:n].copy(), int(out.n_input_points), -1)


def agg_long(agg, values):
    a = np.ascontiguousarray(values, np.int64)
    r = C.c_int64()
    rc = lib().oracle_agg_long(agg, _abi.ptr(a, C.c_int64), len(a), C.byref(r))
    if rc:
        raise RuntimeError(rc)
    return r.value


def agg_double(agg, values):
    a = np.ascontiguousarray(values, np.float64)
    r = C.c_double()
    rc = lib().oracle_agg_double(agg, _abi.ptr(a, C.c_double), len(a), C.byref(r))
    if rc:
        raise RuntimeError(rc)
    return r.value


def compact_rows(rowbatch):
    """rowbatch: opentsdb_amd.compaction.RowBatch -> compaction.RowsResult
    (same placement of the compacted rows as tsdbhip_compact_rows)."""
    from opentsdb_amd import compaction
    desc = rowbatch.fill_desc(_abi.RowsDesc())
    res, out = compaction.out_buffers(rowbatch)
    rc = lib().oracle_compact_rows(C.byref(desc), C.byref(out))
    if rc:
        raise RuntimeError(rc)
    res.n_complex = int(out.n_complex)
    return compaction._trim(res, rowbatch.n_rows)
