"""Host-side packing of compacted KeyValues into the tsdbhip_sg_desc layout.

This is the bridge's job at TsdbQuery.findSpans (TsdbQuery.java:264-266):
every compacted row of every span is copied, byte for byte, into two flat
buffers (qualifiers, values) plus per-row metadata. Rows keep their
reference bytes; only their start offsets are aligned (qualifiers to 8 B,
values to 16 B) so the decode kernel can use wide loads.

The row-acceptance rules of Span.addRow / RowSeq.addRow (Span.java:87-132,
RowSeq.java:92-172) are NOT applied here: the rows are handed over as
scanned, and the library applies the rules itself.
"""
from dataclasses import dataclass, field
import numpy as np

from . import _abi

QUAL_ALIGN = 8
VAL_ALIGN = 16


def _align(x, a):
    return (x + a - 1) // a * a


@dataclass
class KeyValue:
    """One compacted HBase cell as Span.addRow sees it: row-key base_time
    (Bytes.getUnsignedInt(key, metric_width), RowSeq.java:262-264),
    qualifier() and value() bytes."""
    base_time: int
    qualifier: bytes
    value: bytes


@dataclass
class SpanSet:
    """Spans of one SpanGroup, packed (numpy arrays, host memory)."""
    span_row_start: np.ndarray  # uint64 [n_spans+1]
    row_base: np.ndarray        # uint32 [n_rows]
    row_ncells: np.ndarray      # uint32
    row_qual_off: np.ndarray    # uint64
    row_val_off: np.ndarray     # uint64
    row_val_len: np.ndarray     # uint32
    qual_bytes: np.ndarray      # uint8
    val_bytes: np.ndarray       # uint8
    _keep: list = field(default_factory=list, repr=False)

    @property
    def n_spans(self):
        return len(self.span_row_start) - 1

    @property
    def n_rows(self):
        return len(self.row_base)

    def n_cells(self):
        return int(self.row_ncells.astype(np.uint64).sum())

    def fill_desc(self, desc):
        """Point a SgDesc at these arrays (host pointers)."""
        desc.n_spans = self.n_spans
        desc.n_rows = self.n_rows
        desc.span_row_start = _abi.ptr(self.span_row_start, _abi.C.c_uint64)
        desc.row_base = _abi.ptr(self.row_base, _abi.C.c_uint32)
        desc.row_ncells = _abi.ptr(self.row_ncells, _abi.C.c_uint32)
        desc.row_qual_off = _abi.ptr(self.row_qual_off, _abi.C.c_uint64)
        desc.row_val_off = _abi.ptr(self.row_val_off, _abi.C.c_uint64)
        desc.row_val_len = _abi.ptr(self.row_val_len, _abi.C.c_uint32)
        desc.qual_bytes = _abi.ptr(self.qual_bytes, _abi.C.c_uint8)
        desc.qual_nbytes = len(self.qual_bytes)
        desc.val_bytes = _abi.ptr(self.val_bytes, _abi.C.c_uint8)
        desc.val_nbytes = len(self.val_bytes)
        return desc

    def span_rows(self, s):
        """KeyValues of span s (for debugging / host adapters)."""
        out = []
        for r in range(int(self.span_row_start[s]), int(self.span_row_start[s + 1])):
            qo, n = int(self.row_qual_off[r]), int(self.row_ncells[r])
            vo, vl = int(self.row_val_off[r]), int(self.row_val_len[r])
            out.append(KeyValue(int(self.row_base[r]),
                                bytes(self.qual_bytes[qo:qo + 2 * n]),
                                bytes(self.val_bytes[vo:vo + vl])))
        return out

    def shard(self, lo, hi):
        """Spans [lo, hi) as their own SpanSet (offsets kept; buffers shared)."""
        r0, r1 = int(self.span_row_start[lo]), int(self.span_row_start[hi])
        return SpanSet(self.span_row_start[lo:hi + 1] - np.uint64(r0),
                       self.row_base[r0:r1], self.row_ncells[r0:r1],
                       self.row_qual_off[r0:r1], self.row_val_off[r0:r1],
                       self.row_val_len[r0:r1], self.qual_bytes, self.val_bytes)


def pack_spans(spans):
    """spans: list (span order) of lists of KeyValue (row order)."""
    n_rows = sum(len(rows) for rows in spans)
    srs = np.zeros(len(spans) + 1, np.uint64)
    base = np.zeros(n_rows, np.uint32)
    ncells = np.zeros(n_rows, np.uint32)
    qoff = np.zeros(n_rows, np.uint64)
    voff = np.zeros(n_rows, np.uint64)
    vlen = np.zeros(n_rows, np.uint32)
    qparts, vparts = [], []
    qpos = vpos = 0
    r = 0
    for s, rows in enumerate(spans):
        srs[s] = r
        for kv in rows:
            if len(kv.qualifier) % 2:
                raise ValueError("odd qualifier length")
            base[r] = kv.base_time
            ncells[r] = len(kv.qualifier) // 2
            qpos = _align(qpos, QUAL_ALIGN)
            vpos = _align(vpos, VAL_ALIGN)
            qoff[r], voff[r], vlen[r] = qpos, vpos, len(kv.value)
            qparts.append((qpos, kv.qualifier))
            vparts.append((vpos, kv.value))
            qpos += len(kv.qualifier)
            vpos += len(kv.value)
            r += 1
    srs[len(spans)] = r
    qb = np.zeros(_align(max(qpos, 1), 16), np.uint8)
    vb = np.zeros(_align(max(vpos, 1), 16), np.uint8)
    for off, b in qparts:
        qb[off:off + len(b)] = np.frombuffer(b, np.uint8)
    for off, b in vparts:
        vb[off:off + len(b)] = np.frombuffer(b, np.uint8)
    return SpanSet(srs, base, ncells, qoff, voff, vlen, qb, vb)
