"""Synthetic SpanGroups in the exact on-disk encoding of the reference.

Encoders follow the write path (out of scope itself, used here as the
format spec): TSDB.addPoint (TSDB.java:236-352) and
IncomingDataPoints.addPoint (IncomingDataPoints.java:272-286):
  qualifier = (ts - base) << 4 | flags, base = ts - ts % 3600
  long  -> minimal width 1/2/4/8 B (TSDB) or 8 B (IncomingDataPoints), flags len-1
  float -> 4 B, flags 0xB;  double -> 8 B, flags 0xF
A compacted row (CompactionQueue.trivialCompact, CompactionQueue.java:450-474)
is qualifiers concatenated and values concatenated + one 0 meta byte.

`regular()` is bit-identical to the device generator tsdbhip_synth_generate
(splitmix64 keyed by (seed, series, index)); tests check that on the GPU.
"""
import struct
import numpy as np

from . import _abi
from .packing import KeyValue, SpanSet, pack_spans, _align, QUAL_ALIGN, VAL_ALIGN

T0 = 1356998400  # 2013-01-01T00:00Z, divisible by 3600
MAX_TIMESPAN = 3600
FLAG_FLOAT = 0x8

M64 = (1 << 64) - 1
_U = np.uint64


def splitmix64(x):
    """numpy uint64 (vectorized, wrapping)."""
    with np.errstate(over="ignore"):
        z = (x + _U(0x9E3779B97F4A7C15)).astype(np.uint64)
        z = (z ^ (z >> _U(30))) * _U(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> _U(27))) * _U(0x94D049BB133111EB)
        return z ^ (z >> _U(31))


def hash3(seed, s, i):
    with np.errstate(over="ignore"):
        a = splitmix64(_U(seed) ^ (np.asarray(s, np.uint64) * _U(0xD1B54A32D192ED03)))
        return splitmix64(a ^ np.asarray(i, np.uint64))


INV_SD = 1.0 / 37837.0  # Irwin-Hall(4 x U16) standard deviation


def float_value(h):
    """~100 + N(0,1): Irwin-Hall of four 16-bit uniforms; each op one IEEE
    rounding (no FMA) so host and device agree bit for bit."""
    h = np.asarray(h, np.uint64)
    s = ((h & _U(0xFFFF)) + ((h >> _U(16)) & _U(0xFFFF)) +
         ((h >> _U(32)) & _U(0xFFFF)) + ((h >> _U(48)) & _U(0xFFFF))).astype(np.int64) - 131070
    return 100.0 + s.astype(np.float64) * INV_SD


def counter_value(seed, s, i):
    """Monotone counter, increments in (0, 1000): base_s + 500 i + r_i."""
    base = hash3(seed, s, 0xFFFFFFFF) >> _U(24)
    r = hash3(seed, s, i) % _U(500)
    with np.errstate(over="ignore"):
        return (base + _U(500) * np.asarray(i, np.uint64) + r).astype(np.int64)


def regular(n_spans, n_points, kind, seed=1, t0=T0, step=1, span0=0):
    """Regular-cadence SpanGroup (C1/C2/C3 shapes), device-generator layout:
    row R = s * rows_per_span + r, quals at R*qstride, values at R*vstride.
    Series s of this set is global series span0 + s (shards)."""
    if t0 % MAX_TIMESPAN or MAX_TIMESPAN % step:
        raise ValueError("t0 must be hour aligned and step must divide 3600")
    k = MAX_TIMESPAN // step
    rps = (n_points + k - 1) // k
    w = 4 if kind == _abi.SYN_FLOAT32 else 8
    flags = {_abi.SYN_INT64_COUNTER: 0x7, _abi.SYN_FLOAT32: 0xB, _abi.SYN_FLOAT64: 0xF}[kind]
    qstride = _align(2 * k, 16)
    vstride = _align(k * w + 1, 16)
    n_rows = n_spans * rps
    R = np.arange(n_rows, dtype=np.uint64)
    r_in_span = (R % _U(rps)).astype(np.int64)
    span = (R // _U(rps)).astype(np.int64)
    ncells = np.minimum(k, n_points - r_in_span * k).astype(np.uint32)
    base = (t0 + r_in_span * MAX_TIMESPAN).astype(np.uint32)
    qoff = R * _U(qstride)
    voff = R * _U(vstride)
    vlen = np.where(ncells > 1, ncells.astype(np.int64) * w + 1, ncells.astype(np.int64) * w).astype(np.uint32)
    qb = np.zeros(n_rows * qstride, np.uint8)
    vb = np.zeros(n_rows * vstride, np.uint8)
    # all cells
    l_idx = np.repeat(np.arange(n_spans, dtype=np.int64), n_points)
    i_idx = np.tile(np.arange(n_points, dtype=np.int64), n_spans)
    row = l_idx * rps + i_idx // k
    s_idx = l_idx + span0
    c = i_idx % k
    delta = c * step
    q = ((delta << 4) | flags).astype(np.uint16)
    qpos = row * qstride + 2 * c
    qb[qpos] = (q >> 8).astype(np.uint8)
    qb[qpos + 1] = (q & 0xFF).astype(np.uint8)
    if kind == _abi.SYN_INT64_COUNTER:
        v = counter_value(seed, s_idx, i_idx).astype(">i8").view(np.uint8).reshape(-1, 8)
    else:
        fv = float_value(hash3(seed, s_idx, i_idx))
        if kind == _abi.SYN_FLOAT32:
            v = fv.astype(np.float32).astype(">f4").view(np.uint8).reshape(-1, 4)
        else:
            v = fv.astype(">f8").view(np.uint8).reshape(-1, 8)
    vpos = row * vstride + c * w
    for b in range(w):
        vb[vpos + b] = v[:, b]
    srs = np.arange(0, n_rows + 1, rps, dtype=np.uint64)
    return SpanSet(srs, base, ncells, qoff, voff, vlen, qb, vb)


# ---------------------------------------------------------------------------
# KeyValue-level encoders for irregular / mixed test inputs.
def encode_long(value, minimal=True):
    """TSDB.addPoint(long) (minimal width) or IncomingDataPoints (8 B)."""
    if minimal and -128 <= value <= 127:
        v = struct.pack(">b", value)
    elif minimal and -32768 <= value <= 32767:
        v = struct.pack(">h", value)
    elif minimal and -(1 << 31) <= value < (1 << 31):
        v = struct.pack(">i", value)
    else:
        v = struct.pack(">q", value)
    return len(v) - 1, v


def encode_float(value):
    return FLAG_FLOAT | 0x3, struct.pack(">f", value)


def encode_double(value):
    return FLAG_FLOAT | 0x7, struct.pack(">d", value)


def compact_cells(base, cells):
    """cells: list of (ts, flags, value_bytes) all in row `base`, sorted.
    Returns the compacted KeyValue (trivialCompact layout)."""
    q = b"".join(struct.pack(">H", ((ts - base) << 4) | fl) for ts, fl, _ in cells)
    v = b"".join(vb for _, _, vb in cells)
    if len(cells) > 1:
        v += b"\x00"
    return KeyValue(base, q, v)


def series_rows(points):
    """points: list of (ts, flags, value_bytes) sorted by ts -> compacted rows
    (one KeyValue per hour), as TsdbQuery hands them to Span.addRow."""
    rows, cur, cur_base = [], [], None
    for ts, fl, vb in points:
        b = ts - ts % MAX_TIMESPAN
        if cur_base is not None and b != cur_base:
            rows.append(compact_cells(cur_base, cur))
            cur = []
        cur_base = b
        cur.append((ts, fl, vb))
    if cur:
        rows.append(compact_cells(cur_base, cur))
    return rows


def points_int(ts_list, vals, minimal=True):
    out = []
    for t, v in zip(ts_list, vals):
        fl, vb = encode_long(int(v), minimal)
        out.append((int(t), fl, vb))
    return out


def points_float(ts_list, vals, double=False):
    out = []
    for t, v in zip(ts_list, vals):
        fl, vb = encode_double(float(v)) if double else encode_float(float(v))
        out.append((int(t), fl, vb))
    return out


def jittered(n_spans, mean_pts, seed=4, t0=T0, span_range=40_000_000, max_gap=6960,
             float_frac=0.5, float_cell_frac=0.01, minimal=True, rng=None):
    """C4-like input: jittered gaps U{1..max_gap}, variable start/end, half
    float32 series, 1 % float cells in int series. Small sizes only (host)."""
    rng = rng or np.random.default_rng(seed)
    spans = []
    for s in range(n_spans):
        n = max(2, int(rng.integers(mean_pts // 2, mean_pts * 3 // 2 + 1)))
        start = t0 + int(rng.integers(0, max(1, span_range // 4)))
        gaps = rng.integers(1, max_gap + 1, size=n)
        ts = start + np.cumsum(gaps) - gaps[0]
        is_float_series = rng.random() < float_frac
        pts = []
        for j, t in enumerate(ts):
            if is_float_series:
                pts.append((int(t),) + encode_float(float(100 + rng.standard_normal())))
            elif rng.random() < float_cell_frac:
                pts.append((int(t),) + encode_float(float(rng.integers(-1000, 1000)) + 0.5))
            else:
                pts.append((int(t),) + encode_long(int(rng.integers(-10**6, 10**6)), minimal))
        spans.append(series_rows(pts))
    return pack_spans(spans)


def jittered_packed(n_spans, mean_pts, seed=4, t0=T0, span_range=40_000_000, max_gap=6960,
                    float_frac=0.5, float_cell_frac=0.01, absval=False):
    """C4, vectorised: ~mean_pts points per series with
    jittered gaps U{1..max_gap} s from a start in the first quarter of
    `span_range`; `float_frac` of the series float32 (~100 + N(0,1)), the
    others minimal-width longs with `float_cell_frac` float cells. One
    compacted KeyValue per hour row (trivialCompact layout, as series_rows),
    packed like packing.pack_spans (rows 8-B / 16-B aligned). `absval`: the
    same series with |value| (same timestamps and cell types; by convexity a
    lerp of the |y| bounds the |lerp| of the y, so the group's sum over them
    bounds the sum of |terms| a double result is rounded against)."""
    rng = np.random.default_rng(seed)
    n = rng.integers(max(2, mean_pts // 2), mean_pts * 3 // 2 + 1, n_spans).astype(np.int64)
    N = int(n.sum())
    sid = np.repeat(np.arange(n_spans, dtype=np.int64), n)
    first = np.cumsum(n) - n
    gaps = rng.integers(1, max_gap + 1, N).astype(np.int64)
    gaps[first] = 0
    start = t0 + rng.integers(0, max(1, span_range // 4), n_spans).astype(np.int64)
    cs = np.cumsum(gaps)
    ts = start[sid] + cs - cs[first][sid]
    is_fs = rng.random(n_spans) < float_frac
    flt = is_fs[sid] | (rng.random(N) < float_cell_frac)
    fval = np.where(is_fs[sid], 100.0 + rng.standard_normal(N),
                    rng.integers(-1000, 1000, N).astype(np.float64) + 0.5).astype(">f4")
    ival = rng.integers(-10**6, 10**6, N).astype(np.int64)
    if absval:
        fval, ival = np.abs(fval).astype(">f4"), np.abs(ival)
    # minimal long widths (TSDB.java:240-250)
    iw = np.where((ival >= -128) & (ival <= 127), 1,
                  np.where((ival >= -32768) & (ival <= 32767), 2,
                           np.where((ival >= -(1 << 31)) & (ival < (1 << 31)), 4, 8)))
    w = np.where(flt, 4, iw)
    flags = np.where(flt, FLAG_FLOAT | 0x3, w - 1)
    base = ts - ts % MAX_TIMESPAN
    # rows: runs of equal (span, base)
    newrow = np.ones(N, bool)
    newrow[1:] = (sid[1:] != sid[:-1]) | (base[1:] != base[:-1])
    rid = np.cumsum(newrow) - 1
    R = int(rid[-1]) + 1
    rfirst = np.nonzero(newrow)[0]
    rcells = np.diff(np.append(rfirst, N))
    rvraw = np.add.reduceat(w, rfirst)
    rvlen = rvraw + (rcells > 1)
    qlen_al = (2 * rcells + 7) // 8 * 8
    vlen_al = (rvlen + 15) // 16 * 16
    qoff = np.cumsum(qlen_al) - qlen_al
    voff = np.cumsum(vlen_al) - vlen_al
    idx_in_row = np.arange(N) - rfirst[rid]
    qb = np.zeros(int(qlen_al.sum()) + 64, np.uint8)
    q = ((ts - base[rfirst][rid]) << 4) | flags
    qp = qoff[rid] + 2 * idx_in_row
    qb[qp] = (q >> 8).astype(np.uint8)
    qb[qp + 1] = (q & 0xFF).astype(np.uint8)
    wcs = np.cumsum(w) - w
    vpos = voff[rid] + wcs - wcs[rfirst][rid]
    vb = np.zeros(int(vlen_al.sum()) + 64, np.uint8)
    fbytes = fval.view(np.uint8).reshape(N, 4)
    ibytes = ival.astype(">i8").view(np.uint8).reshape(N, 8)
    for width in (1, 2, 4, 8):
        sel = np.nonzero(~flt & (w == width))[0]
        for j in range(width):
            vb[vpos[sel] + j] = ibytes[sel, 8 - width + j]
    sel = np.nonzero(flt)[0]
    for j in range(4):
        vb[vpos[sel] + j] = fbytes[sel, j]
    srs = np.zeros(n_spans + 1, np.uint64)
    srs[1:] = np.cumsum(np.bincount(sid[rfirst], minlength=n_spans))
    return SpanSet(srs, base[rfirst].astype(np.uint32), rcells.astype(np.uint32), qoff.astype(np.uint64),
                   voff.astype(np.uint64), rvlen.astype(np.uint32), qb, vb)
