"""CompactionQueue.compact mirror (secondary path) over tsdbhip_compact_rows.

Reference: src/core/CompactionQueue.java:221-743. For each row (the list of
KeyValues HBase returns for one row key, in qualifier order) the library
computes compacted[0] of compact(row, compacted): the single KV (float-fixed),
the trivialCompact or complexCompact result, nothing, or the exception the
reference throws (IllegalDataException / ArrayIndexOutOfBoundsException).

Batch layout (include/tsdbhip.h, tsdbhip_rows_desc): the qualifiers of a
row's KVs are packed back to back, likewise the values; per KV only the two
u16 lengths travel. `synth_rows` builds the C5 workload of SURVEY.md §8
(1M rows, ~50M cells, mixed widths, legacy floats, pre-compacted cells with
late singles and exact duplicates, a few conflicting duplicates) vectorised
in numpy, with the exact HBase byte encoding.
"""
from dataclasses import dataclass
import ctypes as C

import numpy as np

from . import _abi

NONE, SINGLE, TRIVIAL, COMPLEX, ERROR, OOB = (_abi.ROW_NONE, _abi.ROW_SINGLE, _abi.ROW_TRIVIAL, _abi.ROW_COMPLEX,
                                             _abi.ROW_ERROR, _abi.ROW_OOB)


@dataclass
class RowBatch:
    row_kv_start: np.ndarray  # uint64 [n_rows+1]
    row_qual_off: np.ndarray  # uint64 [n_rows+1]
    row_val_off: np.ndarray   # uint64 [n_rows+1]
    kv_qual_len: np.ndarray   # uint16 [n_kvs]
    kv_val_len: np.ndarray    # uint16 [n_kvs]
    qual_bytes: np.ndarray    # uint8
    val_bytes: np.ndarray     # uint8

    @property
    def n_rows(self):
        return len(self.row_kv_start) - 1

    @property
    def n_kvs(self):
        return len(self.kv_qual_len)

    @property
    def qual_extent(self):
        return int(self.row_qual_off[-1] - self.row_qual_off[0]) if self.n_rows else 0

    @property
    def val_extent(self):
        return int(self.row_val_off[-1] - self.row_val_off[0]) if self.n_rows else 0

    def cell_bytes(self):
        """Input cell bytes (qualifiers + values), SURVEY.md §8(d) for C5."""
        return self.qual_extent + self.val_extent

    def fill_desc(self, d):
        d.flags = 0
        d.n_rows = self.n_rows
        d.n_kvs = self.n_kvs
        d.row_kv_start = _abi.ptr(self.row_kv_start, C.c_uint64)
        d.row_qual_off = _abi.ptr(self.row_qual_off, C.c_uint64)
        d.row_val_off = _abi.ptr(self.row_val_off, C.c_uint64)
        d.kv_qual_len = _abi.ptr(self.kv_qual_len, C.c_uint16)
        d.kv_val_len = _abi.ptr(self.kv_val_len, C.c_uint16)
        d.qual_bytes = _abi.ptr(self.qual_bytes, C.c_uint8)
        d.qual_nbytes = len(self.qual_bytes)
        d.val_bytes = _abi.ptr(self.val_bytes, C.c_uint8)
        d.val_nbytes = len(self.val_bytes)
        return d


def pack_rows(rows):
    """rows: list of lists of (qualifier bytes, value bytes), each row in the
    order HBase returns its KVs."""
    n_kvs = sum(len(r) for r in rows)
    rks = np.zeros(len(rows) + 1, np.uint64)
    rqo = np.zeros(len(rows) + 1, np.uint64)
    rvo = np.zeros(len(rows) + 1, np.uint64)
    ql = np.zeros(n_kvs, np.uint16)
    vl = np.zeros(n_kvs, np.uint16)
    qparts, vparts = [], []
    k = qpos = vpos = 0
    for r, row in enumerate(rows):
        rks[r], rqo[r], rvo[r] = k, qpos, vpos
        for q, v in row:
            if len(q) > 0xFFFF or len(v) > 0xFFFF:
                raise ValueError("KeyValue longer than 65535 bytes: not an OpenTSDB cell")
            ql[k], vl[k] = len(q), len(v)
            qparts.append(q)
            vparts.append(v)
            qpos += len(q)
            vpos += len(v)
            k += 1
    rks[-1], rqo[-1], rvo[-1] = k, qpos, vpos
    qb = np.zeros(qpos + 64, np.uint8)
    vb = np.zeros(vpos + 64, np.uint8)
    qb[:qpos] = np.frombuffer(b"".join(qparts), np.uint8)
    vb[:vpos] = np.frombuffer(b"".join(vparts), np.uint8)
    return RowBatch(rks, rqo, rvo, ql, vl, qb, vb)


@dataclass
class RowsResult:
    status: np.ndarray    # uint8 [n_rows]
    qual_off: np.ndarray  # uint64
    qual_len: np.ndarray  # uint32
    val_off: np.ndarray   # uint64
    val_len: np.ndarray   # uint32
    qual: np.ndarray      # uint8 (rows placed per tsdbhip.h; gaps undefined)
    val: np.ndarray
    write: np.ndarray = None    # uint8 [n_rows]: tsdb.put of the compacted cell
    keep_kv: np.ndarray = None  # int32 [n_rows]: KV (index in the row) not to delete, -1 none
    n_complex: int = 0

    def row(self, r):
        """-> (status, qualifier bytes, value bytes) of row r."""
        qo, vo = int(self.qual_off[r]), int(self.val_off[r])
        return (int(self.status[r]), bytes(self.qual[qo:qo + int(self.qual_len[r])]),
                bytes(self.val[vo:vo + int(self.val_len[r])]))

    def rows(self):
        return [self.row(r) for r in range(len(self.status))]

    def decision(self, r, kv_qual_lens):
        """-> (put?, sorted KV indices to delete) of row r, the flush-path
        writes of CompactionQueue.compact (CompactionQueue.java:419-434) for a
        row old enough to be written back; kv_qual_lens = the row's KV
        qualifier lengths."""
        if int(self.status[r]) not in (TRIVIAL, COMPLEX):
            return False, []
        keep = int(self.keep_kv[r])
        dele = [i for i, ql in enumerate(kv_qual_lens) if ql and ql % 2 == 0 and i != keep]
        return bool(self.write[r]), dele

    @staticmethod
    def _packed(buf, off, ln):
        ln = ln.astype(np.int64)
        tot = int(ln.sum())
        if tot == 0:
            return np.zeros(0, np.uint8)
        starts = np.cumsum(ln) - ln
        idx = np.repeat(off.astype(np.int64) - starts, ln) + np.arange(tot, dtype=np.int64)
        return buf[idx]

    def packed_qual(self):
        """All compacted qualifiers concatenated in row order."""
        return self._packed(self.qual, self.qual_off, self.qual_len)

    def packed_val(self):
        return self._packed(self.val, self.val_off, self.val_len)


def out_buffers(batch: RowBatch):
    n = batch.n_rows
    qcap = batch.qual_extent + 64
    vcap = batch.val_extent + n + 64
    res = RowsResult(np.zeros(max(n, 1), np.uint8), np.zeros(max(n, 1), np.uint64),
                     np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.uint64),
                     np.zeros(max(n, 1), np.uint32), np.zeros(qcap, np.uint8), np.zeros(vcap, np.uint8),
                     np.full(max(n, 1), 0xEE, np.uint8), np.full(max(n, 1), -7, np.int32))
    out = _abi.RowsOut(qual_capacity=qcap, val_capacity=vcap,
                       row_status=_abi.ptr(res.status, C.c_uint8),
                       row_qual_off=_abi.ptr(res.qual_off, C.c_uint64),
                       row_qual_len=_abi.ptr(res.qual_len, C.c_uint32),
                       row_val_off=_abi.ptr(res.val_off, C.c_uint64),
                       row_val_len=_abi.ptr(res.val_len, C.c_uint32),
                       qual_bytes=_abi.ptr(res.qual, C.c_uint8),
                       val_bytes=_abi.ptr(res.val, C.c_uint8),
                       row_write=_abi.ptr(res.write, C.c_uint8),
                       row_keep_kv=_abi.ptr(res.keep_kv, C.c_int32))
    return res, out


def _trim(res, n):
    for f in ("status", "qual_off", "qual_len", "val_off", "val_len", "write", "keep_kv"):
        setattr(res, f, getattr(res, f)[:n])
    return res


def compact_rows(ctx, batch: RowBatch) -> RowsResult:
    """tsdbhip_compact_rows on the GPU (host buffers in and out)."""
    d = batch.fill_desc(_abi.RowsDesc())
    res, out = out_buffers(batch)
    ctx.check(ctx._lib.tsdbhip_compact_rows(ctx.handle, C.byref(d), C.byref(out)))
    res.n_complex = int(out.n_complex)
    return _trim(res, batch.n_rows)


# --------------------------------------------------------------------------
# C5 synthetic workload: exact HBase encoding of
#  * single cells written by TSDB.addPoint (TSDB.java:240-250,285,321,342-346):
#    2-byte qualifier (delta << 4 | flags), BE value of 1/2/4/8 bytes (long)
#    or 4/8 bytes (float/double);
#  * legacy floats: flags 0x?B with an 8-byte value 00000000 || float bits
#    (fixed by fixFloatingPointValue, CompactionQueue.java:510-544);
#  * longs whose flags claim 4 bytes but hold 8 (fixQualifierFlags :490-499);
#  * compacted cells (trivialCompact layout :450-474: qualifiers || values ||
#    0x00) over a prefix of the row's points, followed by late single cells,
#    exact duplicates of compacted points and, rarely, conflicting ones;
#  * junk KVs with an odd-length qualifier (skipped, :301-306).
# KVs of a row are ordered as HBase returns them: by qualifier bytes,
# unsigned, a shorter prefix first (Bytes.memcmp).
# --------------------------------------------------------------------------
# cell kinds: (flags, raw value length, fixed flags, fixed length)
_KINDS = np.array([
    (0x0, 1, 0x0, 1), (0x1, 2, 0x1, 2), (0x3, 4, 0x3, 4), (0x7, 8, 0x7, 8),   # longs
    (0xB, 4, 0xB, 4), (0xF, 8, 0xF, 8),                                       # float, double
    (0xB, 8, 0xB, 4),                                                         # legacy float
    (0x3, 8, 0x7, 8),                                                         # wrong-length long
], np.int64)
_KIND_P = np.array([0.22, 0.18, 0.18, 0.18, 0.12, 0.10, 0.01, 0.01])


def synth_rows(n_rows, seed=5, min_cells=1, max_cells=99, p_complex=0.10, p_conflict=0.001,
               p_junk=0.001, p_dup=0.2, kind_p=None):
    """C5: n_rows rows with U{min..max} points each; returns a RowBatch."""
    rng = np.random.default_rng(seed)
    n = rng.integers(min_cells, max_cells + 1, n_rows).astype(np.int64)
    N = int(n.sum())
    cstart = np.cumsum(n) - n
    crow = np.repeat(np.arange(n_rows, dtype=np.int64), n)
    cidx = np.arange(N, dtype=np.int64) - cstart[crow]
    # distinct sorted deltas per row: sorted U[0, 3600-n] + rank, the sorted
    # uniforms drawn as normalised exponential spacings (no sort needed)
    ext = n + 1
    es = np.cumsum(ext) - ext
    cs = np.cumsum(rng.exponential(size=int(ext.sum())))
    lo = np.where(es > 0, cs[np.maximum(es - 1, 0)], 0.0)
    tot = cs[es + n] - lo
    pos = np.repeat(es, n) + cidx
    uu = (cs[pos] - lo[crow]) / tot[crow]
    delta = np.minimum((uu * (3601 - n[crow])).astype(np.int64), 3600 - n[crow]) + cidx
    kind = rng.choice(len(_KINDS), N, p=_KIND_P if kind_p is None else kind_p)
    kk = _KINDS[kind]
    rflag, rlen, fflag, flen = kk[:, 0], kk[:, 1], kk[:, 2], kk[:, 3]
    rq = (delta << 4) | rflag
    fq = (delta << 4) | fflag
    # raw value bytes; a fixed value is the raw value minus a legacy prefix
    rvoff = np.cumsum(rlen) - rlen
    rv = rng.integers(0, 256, int(rlen.sum()), dtype=np.uint8)
    legacy = kind == 6
    for j in range(4):
        rv[rvoff[legacy] + j] = 0
    fvoff = rvoff + (rlen - flen)

    # row types
    rtype = np.zeros(n_rows, np.int64)                    # 0 plain singles
    x = rng.random(n_rows)
    rtype[(x < p_complex) & (n >= 2)] = 1                 # compacted prefix + singles
    rtype[(x < p_conflict) & (n >= 2)] = 2                # ... plus a conflicting dup
    junk = rng.random(n_rows) < p_junk
    k = np.where(rtype > 0, (rng.random(n_rows) * (n - 1)).astype(np.int64) + 2, 0)  # U{2..n}
    in_prefix = cidx < k[crow]
    # KVs: singles (cells outside a compacted prefix, or exact duplicates),
    # one compacted KV per complex row, conflicting duplicates, junk.
    dup = in_prefix & (rng.random(N) < p_dup)
    single_cells = np.nonzero(~in_prefix | dup)[0]
    comp_rows = np.nonzero(rtype > 0)[0]
    conf_rows = np.nonzero(rtype == 2)[0]
    conf_cells = cstart[conf_rows] + (rng.random(len(conf_rows)) * k[conf_rows]).astype(np.int64)
    conf_cells = conf_cells[~dup[conf_cells]]  # keep the row's singles strictly increasing
    junk_rows = np.nonzero(junk)[0]

    # KV table: type 0 single(raw), 1 compacted, 2 conflicting single, 3 junk
    kv_type = np.concatenate([np.zeros(len(single_cells), np.int64), np.ones(len(comp_rows), np.int64),
                              np.full(len(conf_cells), 2, np.int64), np.full(len(junk_rows), 3, np.int64)])
    kv_row = np.concatenate([crow[single_cells], comp_rows, crow[conf_cells], junk_rows])
    kv_cell = np.concatenate([single_cells, cstart[comp_rows], conf_cells, np.zeros(len(junk_rows), np.int64)])
    kv_ncell = np.where(kv_type == 1, k[kv_row], 1)
    kv_key = np.where(kv_type == 1, fq[kv_cell], rq[kv_cell])
    kv_key = np.where(kv_type == 3, 0x10000, kv_key)  # junk '\xff' sorts last
    kv_qlen = np.where(kv_type == 3, 1, 2 * kv_ncell)
    order = np.argsort((kv_row << 26) | (kv_key << 9) | kv_qlen, kind="stable")
    kv_type, kv_row, kv_cell, kv_ncell, kv_qlen = (a[order] for a in (kv_type, kv_row, kv_cell, kv_ncell, kv_qlen))
    n_kvs = len(kv_type)

    # qualifier stream: one 2-byte piece per cell entry (junk: 1 byte 0xFF)
    n_ent = np.where(kv_type == 3, 1, kv_ncell)
    ent_kv = np.repeat(np.arange(n_kvs, dtype=np.int64), n_ent)
    ent_start = np.cumsum(n_ent) - n_ent
    ent_cell = kv_cell[ent_kv] + (np.arange(len(ent_kv), dtype=np.int64) - ent_start[ent_kv])
    et = kv_type[ent_kv]
    eq = np.where(et == 1, fq[ent_cell], rq[ent_cell])
    qpair = np.stack([(eq >> 8) & 0xFF, eq & 0xFF], axis=1).astype(np.uint8)
    qmask = np.ones((len(ent_kv), 2), bool)
    qmask[et == 3, 1] = False
    qpair[et == 3, 0] = 0xFF
    qual = qpair[qmask]

    # value stream: raw value (singles), fixed values + 0x00 (compacted),
    # flipped last byte (conflicts), 2 random bytes (junk)
    e_len = np.where(et == 1, flen[ent_cell], rlen[ent_cell])
    e_len = np.where(et == 3, 2, e_len)
    e_src = np.where(et == 1, fvoff[ent_cell], rvoff[ent_cell])
    e_src = np.where(et == 3, 0, e_src)
    is_last_ent = np.zeros(len(ent_kv), bool)
    is_last_ent[np.cumsum(n_ent) - 1] = True
    term = (et == 1) & is_last_ent
    tot = int(e_len.sum() + term.sum())
    # output position of each entry's first byte, with room for terminators
    e_out = np.cumsum(e_len + term) - (e_len + term)
    val = np.zeros(tot, np.uint8)
    idx_out = np.repeat(e_out - (np.cumsum(e_len) - e_len), e_len) + np.arange(int(e_len.sum()), dtype=np.int64)
    idx_src = np.repeat(e_src - (np.cumsum(e_len) - e_len), e_len) + np.arange(int(e_len.sum()), dtype=np.int64)
    val[idx_out] = rv[idx_src]
    conf_last = e_out[et == 2] + e_len[et == 2] - 1
    val[conf_last] ^= 0x5A
    kv_vlen = np.bincount(ent_kv, weights=e_len + term, minlength=n_kvs).astype(np.int64)

    def per_row(w):
        return np.bincount(kv_row + 1, weights=w, minlength=n_rows + 1).astype(np.int64)

    rk = np.cumsum(per_row(None)).astype(np.uint64)
    qsum = per_row(kv_qlen)
    vsum = per_row(kv_vlen)
    qb = np.zeros(len(qual) + 64, np.uint8)
    qb[:len(qual)] = qual
    vb = np.zeros(tot + 64, np.uint8)
    vb[:tot] = val
    return RowBatch(rk, np.cumsum(qsum).astype(np.uint64), np.cumsum(vsum).astype(np.uint64),
                    kv_qlen.astype(np.uint16), kv_vlen.astype(np.uint16), qb, vb)
