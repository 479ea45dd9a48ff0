"""k_decode_rows (k_decode.hip): spans of many short rows (C4's shape: ~one
cell per hourly row) decoded a thread per row, when the span's E is its
accepted cells in order; otherwise the block's first wave walks the span as
k_decode_nods does. Against the oracle (RowSeq.java:360-497, Span.java:87-132
row assembly, SpanGroup.java:510-784): dropped rows, merged rows, illegal
widths raised at their lazy index, windows that start inside the spans (the
walk), NaN results."""
import numpy as np
import pytest

from helpers import T0, U32MAX, assert_same, corrupt_qual, run_both
from opentsdb_amd import _abi, synth

AGGS = [0, 1, 2, 3, 4]


def sparse(seed, float_frac=0.5):
    # gaps up to 30000 s: most hourly rows hold one cell, some two or more
    return synth.jittered(12, 300, seed=seed, span_range=9_000_000, max_gap=30_000, float_frac=float_frac)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_many_short_rows(ctx, seed, agg, rate):
    ss = sparse(seed)
    assert len(ss.row_base) >= 64 * 12
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    g, o = run_both(ctx, ss, agg=agg, rate=rate, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 4])
def test_many_short_rows_int(ctx, agg):
    """integer spans: the long outputs bit-exact; the double ones (dev, and
    the lerped-to-double points) at 1e-9 in the default merge order, bit-exact
    under EXACT_ORDER"""
    ss = sparse(3, float_frac=0.0)
    g, o = run_both(ctx, ss, agg=agg)
    assert_same(g, o)
    g, o = run_both(ctx, ss, agg=agg, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.gpu
def test_window_inside_the_spans(ctx):
    """start after the spans' first points: those spans take the walk"""
    ss = sparse(4)
    lo = int(ss.row_base.min())
    for start, end in ((lo + 2_000_000, U32MAX), (0, lo + 5_000_000), (lo + 1_000_000, lo + 6_000_000)):
        g, o = run_both(ctx, ss, start=start, end=end, agg=0)
        assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("row", [0, 37, 150])
def test_illegal_width_in_a_middle_row(ctx, row):
    """a 3-byte int qualifier (IllegalDataException, RowSeq.java:203): the
    error's lazy output index from the row-parallel decode"""
    ss = corrupt_qual(sparse(5, float_frac=0.0), 7, 0, lambda q: (q & ~0xF) | 0x2, row=row)
    g, o = run_both(ctx, ss, agg=0)
    assert o.code == _abi.E_ILLEGAL_DATA
    assert_same(g, o)
