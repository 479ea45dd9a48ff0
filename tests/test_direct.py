"""The no-downsampling direct path (opentsdb_amd/csrc/k_direct.hip): spans on a
regular cadence whose points are consecutive union-grid ranks are reduced
straight from the reference's value bytes. Each case is checked against the
oracle with the path forced on (ctx option decode=direct) and in auto mode;
cases that break a precondition (phase shift, mixed cadences, points after
end, mixed types, start at a row boundary) check that the fallback to the E
path is exact too. Integers bit-exact, doubles 1e-9 rel. (helpers.py)."""
import numpy as np
import pytest

from helpers import with_option, I, F, T0, U32MAX, run_both, assert_same
from opentsdb_amd import _abi, packing, synth

pytestmark = pytest.mark.gpu

AGGS = [0, 1, 2, 3, 4]


@pytest.fixture(autouse=True, params=["auto", "direct"])
def path(request):
    yield from with_option(request, "decode", request.param, "auto")


def long_series(ts, vals):
    return I([(int(t), int(v)) for t, v in zip(ts, vals)], minimal=False)


def cadence(n_spans, n_pts, step, seed, offsets=None, phase=None, lo=-10**6, hi=10**6):
    """int64 spans at `step`, span s starting offsets[s] steps after T0 and
    shifted by phase[s] seconds"""
    rng = np.random.default_rng(seed)
    spans = []
    for s in range(n_spans):
        o = 0 if offsets is None else offsets[s]
        p = 0 if phase is None else phase[s]
        ts = T0 + p + step * (o + np.arange(n_pts))
        spans.append(long_series(ts, rng.integers(lo, hi, n_pts)))
    return packing.pack_spans(spans)


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_same_cadence_staggered_starts(ctx, agg, rate):
    ss = cadence(37, 300, 10, seed=agg, offsets=[(7 * s) % 50 for s in range(37)])
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_regular_generator_shapes(ctx, agg, rate):
    """synth.regular: one hourly row per span (C3) and three rows per span."""
    for n_pts, step in [(3600, 1), (1000, 10)]:
        ss = synth.regular(20, n_pts, _abi.SYN_INT64_COUNTER, seed=5, step=step)
        g, o = run_both(ctx, ss, agg=agg, rate=rate)
        assert_same(g, o)


@pytest.mark.parametrize("kind", [_abi.SYN_FLOAT32, _abi.SYN_FLOAT64])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_float_spans(ctx, kind, agg, rate):
    ss = synth.regular(16, 900, kind, seed=2, step=10)
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    g, o = run_both(ctx, ss, agg=agg, rate=rate, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("agg", AGGS)
def test_mixed_int_and_float_spans(ctx, agg):
    """int64, float32 and float64 spans on one cadence: the dual path; a float
    span starting later forces the double path before it (Q3)."""
    rng = np.random.default_rng(agg)
    spans = []
    for s in range(12):
        ts = T0 + 10 * ((3 * s) % 20 + np.arange(200))
        if s % 3 == 0:
            spans.append(long_series(ts, rng.integers(-1000, 1000, 200)))
        else:
            spans.append(F([(int(t), float(v) / 8) for t, v in zip(ts, rng.integers(-80, 80, 200))], double=s % 3 == 2))
    ss = packing.pack_spans(spans)
    for rate in (False, True):
        g, o = run_both(ctx, ss, agg=agg, rate=rate)
        assert_same(g, o)


@pytest.mark.parametrize("agg", [0, 2, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_phase_shift_falls_back(ctx, agg, rate):
    """Spans 5 s out of phase interleave on the grid: every one needs lerps."""
    ss = cadence(10, 150, 10, seed=3, phase=[5 * (s % 2) for s in range(10)])
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)


@pytest.mark.parametrize("agg", [0, 1, 3, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_mixed_cadences(ctx, agg, rate):
    """10 s and 20 s spans in phase: the 20 s ones skip grid points (lerp)."""
    rng = np.random.default_rng(11)
    spans = []
    for s in range(9):
        step = 20 if s % 3 == 1 else 10
        n = 120 if step == 10 else 60
        spans.append(long_series(T0 + step * np.arange(n), rng.integers(-500, 500, n)))
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)


@pytest.mark.parametrize("rate", [False, True])
def test_window_start_at_row_boundary_and_end(ctx, rate):
    """start at an hour boundary inside a 3-row span (no Q1: the seek lands on
    a row start) takes the direct path with E[0] in row 2; an end inside the
    spans leaves points after end (lerp brackets) to the E path."""
    ss = synth.regular(8, 1000, _abi.SYN_INT64_COUNTER, seed=9, step=10)
    for start, end in [(T0 + 7200, U32MAX), (0, T0 + 5000), (T0 + 3600, T0 + 8000), (T0 + 9000, U32MAX)]:
        for agg in (0, 2, 4):
            g, o = run_both(ctx, ss, start=start, end=end, agg=agg, rate=rate)
            assert_same(g, o)


def test_single_point_and_int32_rows(ctx):
    """one-point spans (no cadence), 4-byte ints (minimal width of small
    values stays 4 B only when forced), and a wide-value span."""
    spans = [long_series([T0 + 100], [5]), long_series(T0 + 100 + 10 * np.arange(30), np.arange(30)),
             I([(T0 + 100 + 10 * i, 70000 + i) for i in range(30)])]  # minimal: 4-byte ints
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        for rate in (False, True):
            g, o = run_both(ctx, ss, agg=agg, rate=rate)
            assert_same(g, o)


def test_many_spans_chunked_reduce(ctx):
    """enough spans for several span chunks per tile and runs of direct spans
    interrupted by fallback spans"""
    n = 1500
    rng = np.random.default_rng(21)
    spans = []
    for s in range(n):
        ph = 5 if s % 97 == 0 else 0
        ts = T0 + ph + 10 * ((s % 13) + np.arange(80))
        spans.append(long_series(ts, rng.integers(-10**12, 10**12, 80)))
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        for rate in (False, True):
            g, o = run_both(ctx, ss, agg=agg, rate=rate)
            assert_same(g, o)


def test_integer_dev_batches(ctx):
    """integer dev without rate reduces in one span-ordered pass
    (Aggregators.java:196-217) over direct spans: 4- and 8-byte cells,
    staggered starts and ends (lanes where a span is inactive), a batch of 64
    spans cut by a fallback span, a span count that is not a multiple of 64"""
    rng = np.random.default_rng(5)
    spans = []
    for s in range(333):
        a = (s * 7) % 40
        n = 600 - (s * 11) % 50
        ts = T0 + 10 * (a + np.arange(n))
        if s % 3 == 0:  # minimal widths: 4-byte cells
            v = rng.integers(2**20, 2**30, n) * rng.choice([-1, 1], n)  # (every cell 4 bytes wide)
            spans.append(I([(int(t), int(x)) for t, x in zip(ts, v)]))
        elif s == 200:  # a phase shift: this batch takes the general path
            spans.append(long_series(ts + 3, rng.integers(-10**15, 10**15, n)))
        else:
            spans.append(long_series(ts, rng.integers(-10**15, 10**15, n)))
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss, agg=4)
    assert_same(g, o)
