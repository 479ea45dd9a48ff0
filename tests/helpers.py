"""Shared test helpers: build SpanGroups, run GPU and oracle, compare."""
import numpy as np

import oracle
from opentsdb_amd import _abi, core, synth, packing

T0 = synth.T0
U32MAX = (1 << 32) - 1


def I(pts, minimal=True):
    """int series rows from [(ts, value)]"""
    return synth.series_rows(synth.points_int([p[0] for p in pts], [p[1] for p in pts], minimal))


def F(pts, double=False):
    return synth.series_rows(synth.points_float([p[0] for p in pts], [p[1] for p in pts], double))


def M(pts):
    """mixed series rows from [(ts, value)] — python int -> long, float -> float32"""
    out = []
    for t, v in pts:
        if isinstance(v, float):
            out.append((t,) + synth.encode_float(v))
        else:
            out.append((t,) + synth.encode_long(v))
    return synth.series_rows(out)


def run_both(ctx, spanset, start=0, end=U32MAX, agg=0, rate=False, ds_interval=0, ds_agg=0, exact=False):
    g = core.run_spanset(ctx, spanset, start, end, agg, rate, ds_interval, ds_agg, exact=exact)
    o = oracle.spangroup(spanset, start, end, agg, rate, ds_interval, ds_agg)
    return g, o


def assert_same(g, o, rtol=1e-9, exact_double=False, check_err_index=True, abs_scale=None):
    """Integers and timestamps bit-exact; doubles at `rtol` relative to the
    result, or, with `abs_scale` (per output point: the same aggregation over
    |terms|, for mixed-sign sums where the result itself can cancel to ~0,
    SURVEY.md §8(d)), |gpu - oracle| <= rtol * abs_scale."""
    rc, ts, isi, bits, n_in, err_at = g
    assert rc == o.code, f"code gpu={_abi.ERR_NAMES.get(rc, rc)} oracle={_abi.ERR_NAMES.get(o.code, o.code)}"
    assert n_in == o.n_input_points, f"aggregatedSize gpu={n_in} oracle={o.n_input_points}"
    if rc == 0 or check_err_index:
        assert len(ts) == len(o.ts), f"n_out gpu={len(ts)} oracle={len(o.ts)}"
    n = min(len(ts), len(o.ts))
    np.testing.assert_array_equal(ts[:n], o.ts[:n], err_msg="timestamps")
    np.testing.assert_array_equal(isi[:n], o.is_int[:n], err_msg="isInteger")
    ints = o.is_int[:n].astype(bool)
    np.testing.assert_array_equal(bits[:n][ints], o.bits[:n][ints], err_msg="long values")
    gd = bits[:n][~ints].view(np.float64)
    od = o.bits[:n][~ints].view(np.float64)
    if exact_double:
        np.testing.assert_array_equal(bits[:n][~ints], o.bits[:n][~ints], err_msg="double bits")
    elif abs_scale is not None:
        sc = np.asarray(abs_scale)[:n][~ints]
        err = np.abs(gd - od)
        bad = ~(err <= rtol * sc)
        assert not bad.any(), (f"double values: {int(bad.sum())} of {len(gd)} beyond {rtol} x sum|terms|; first at "
                               f"{int(np.nonzero(bad)[0][0])}: err {err[bad][0]!r}, sum|terms| {sc[bad][0]!r}")
    else:
        np.testing.assert_allclose(gd, od, rtol=rtol, atol=0, err_msg="double values")


def corrupt_qual(ss, span, cell, fn, row=0):
    """A copy of the SpanSet with one qualifier (cell `cell` of row `row` of
    span `span`) rewritten by fn(q) -> q' (16-bit host-order values)."""
    qb = ss.qual_bytes.copy()
    r = int(ss.span_row_start[span]) + row
    off = int(ss.row_qual_off[r]) + 2 * cell
    q = (int(qb[off]) << 8) | int(qb[off + 1])
    q2 = fn(q) & 0xFFFF
    qb[off], qb[off + 1] = q2 >> 8, q2 & 0xFF
    return packing.SpanSet(ss.span_row_start, ss.row_base, ss.row_ncells, ss.row_qual_off, ss.row_val_off,
                           ss.row_val_len, qb, ss.val_bytes)


def with_option(request, name, value, default):
    """Fixture body: set a context option (tsdbhip_set_option) for a GPU test
    and restore its default after it; CPU tests open no context."""
    if request.node.get_closest_marker("gpu") is None:
        yield value
        return
    c = request.getfixturevalue("ctx")
    c.set_option(name, value)
    try:
        yield value
    finally:
        c.set_option(name, default)
