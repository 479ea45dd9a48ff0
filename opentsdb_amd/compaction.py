"""CompactionQueue.compact mirror (secondary path) over tsdbhip_compact_rows.

Reference: src/core/CompactionQueue.java:221-743. For each row (the list of
KeyValues HBase returns for one row key, in order) the library computes
compacted[0] of compact(row, compacted): the single KV (float-fixed), the
trivialCompact or complexCompact result, nothing, or an IllegalDataException.
"""
from dataclasses import dataclass, field
import ctypes as C

import numpy as np

from . import _abi
from .packing import _align


@dataclass
class RowBatch:
    row_kv_start: np.ndarray  # uint64 [n_rows+1]
    kv_qual_off: np.ndarray   # uint64
    kv_qual_len: np.ndarray   # uint32
    kv_val_off: np.ndarray    # uint64
    kv_val_len: np.ndarray    # uint32
    qual_bytes: np.ndarray    # uint8
    val_bytes: np.ndarray     # uint8

    @property
    def n_rows(self):
        return len(self.row_kv_start) - 1

    @property
    def n_kvs(self):
        return len(self.kv_qual_len)

    def fill_desc(self, d):
        d.flags = 0
        d.n_rows = self.n_rows
        d.n_kvs = self.n_kvs
        d.row_kv_start = _abi.ptr(self.row_kv_start, C.c_uint64)
        d.kv_qual_off = _abi.ptr(self.kv_qual_off, C.c_uint64)
        d.kv_qual_len = _abi.ptr(self.kv_qual_len, C.c_uint32)
        d.kv_val_off = _abi.ptr(self.kv_val_off, C.c_uint64)
        d.kv_val_len = _abi.ptr(self.kv_val_len, C.c_uint32)
        d.qual_bytes = _abi.ptr(self.qual_bytes, C.c_uint8)
        d.qual_nbytes = len(self.qual_bytes)
        d.val_bytes = _abi.ptr(self.val_bytes, C.c_uint8)
        d.val_nbytes = len(self.val_bytes)
        return d


def pack_rows(rows):
    """rows: list of lists of (qualifier bytes, value bytes)."""
    n_kvs = sum(len(r) for r in rows)
    rks = np.zeros(len(rows) + 1, np.uint64)
    qo = np.zeros(n_kvs, np.uint64)
    ql = np.zeros(n_kvs, np.uint32)
    vo = np.zeros(n_kvs, np.uint64)
    vl = np.zeros(n_kvs, np.uint32)
    qparts, vparts = [], []
    qpos = vpos = 0
    k = 0
    for r, row in enumerate(rows):
        rks[r] = k
        for q, v in row:
            qpos = _align(qpos, 2)
            qo[k], ql[k], vo[k], vl[k] = qpos, len(q), vpos, len(v)
            qparts.append((qpos, q))
            vparts.append((vpos, v))
            qpos += len(q)
            vpos += len(v)
            k += 1
    rks[len(rows)] = k
    qb = np.zeros(_align(qpos + 16, 16), np.uint8)
    vb = np.zeros(_align(vpos + 16, 16), np.uint8)
    for off, b in qparts:
        qb[off:off + len(b)] = np.frombuffer(b, np.uint8)
    for off, b in vparts:
        vb[off:off + len(b)] = np.frombuffer(b, np.uint8)
    return RowBatch(rks, qo, ql, vo, vl, qb, vb)


def compact_rows(ctx, batch: RowBatch):
    """-> list of (status, qualifier bytes, value bytes) per row."""
    d = batch.fill_desc(_abi.RowsDesc())
    n = batch.n_rows
    qcap = len(batch.qual_bytes) + 16
    vcap = len(batch.val_bytes) + 16 + n
    st = np.zeros(max(n, 1), np.uint8)
    qo = np.zeros(max(n, 1), np.uint64)
    ql = np.zeros(max(n, 1), np.uint32)
    vo = np.zeros(max(n, 1), np.uint64)
    vl = np.zeros(max(n, 1), np.uint32)
    qb = np.zeros(qcap, np.uint8)
    vb = np.zeros(vcap, np.uint8)
    out = _abi.RowsOut(qual_capacity=qcap, val_capacity=vcap,
                       row_status=_abi.ptr(st, C.c_uint8), row_qual_off=_abi.ptr(qo, C.c_uint64),
                       row_qual_len=_abi.ptr(ql, C.c_uint32), row_val_off=_abi.ptr(vo, C.c_uint64),
                       row_val_len=_abi.ptr(vl, C.c_uint32), qual_bytes=_abi.ptr(qb, C.c_uint8),
                       val_bytes=_abi.ptr(vb, C.c_uint8))
    ctx.check(ctx._lib.tsdbhip_compact_rows(ctx.handle, C.byref(d), C.byref(out)))
    return [(int(st[r]), bytes(qb[int(qo[r]):int(qo[r]) + int(ql[r])]),
             bytes(vb[int(vo[r]):int(vo[r]) + int(vl[r])])) for r in range(n)]
