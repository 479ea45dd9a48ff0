"""k_ds_reg's aligned-group reduction (FapArgs in k_ds_reg.hip): when every
kept span of a downsampled integer group has the same first timestamp,
cadence and length (C3*: series written in lockstep), the per-span bucket
sequences coincide, G is that sequence and every span is active at every t
(SpanGroup.java:510-608), so the cross-series aggregate at G[b] is the
combine of bucket b over the spans, exact in any order for wrapping sums and
min / max (Aggregators.java:76-180); blocks combine their spans' buckets and
no E is written. Groups that look aligned (same first / last timestamp) but
hold a span outside the class are rerun with E (timing.paths tells which
ran). Every result is compared with the oracle bit-exactly."""
import numpy as np
import pytest

from helpers import I, F, T0, U32MAX, assert_same, run_both
from opentsdb_amd import _abi, core, packing, synth

pytestmark = pytest.mark.gpu
I64 = _abi.SYN_INT64_COUNTER


def paths(ctx):
    return ctx.timing().paths


@pytest.mark.parametrize("agg", [0, 1, 2, 3])
@pytest.mark.parametrize("dsa", [0, 1, 2, 3])
def test_aligned_group_taken(ctx, agg, dsa):
    ss = synth.regular(300, 3600, I64, seed=11, step=1)
    g, o = run_both(ctx, ss, 0, U32MAX, agg, False, 60, dsa)
    assert_same(g, o)
    assert paths(ctx) & _abi.PATH_ALIGNED_GROUP


@pytest.mark.parametrize("step,interval", [(1, 60), (10, 60), (8, 100), (60, 60), (1, 3600)])
def test_aligned_group_cadences(ctx, step, interval):
    """bucket sizes kk = ceil(interval / step), a partial last bucket, a
    bucket per point, one bucket per span"""
    n = 3600 // step
    ss = synth.regular(97, n - 3, I64, seed=3, step=step)
    g, o = run_both(ctx, ss, 0, U32MAX, 0, False, interval, 3)
    assert_same(g, o)
    if n - 3 >= 64:  # (rows of fewer cells take the general decode kernel)
        assert paths(ctx) & _abi.PATH_ALIGNED_GROUP


def test_end_inside_the_group(ctx):
    """end cuts the bucket sequence: G holds the buckets <= end; the spans
    stay active (their last points lie after end)"""
    ss = synth.regular(64, 3600, I64, seed=5, step=1)
    for end in (T0 + 1000, T0 + 29, T0 + 3599):
        g, o = run_both(ctx, ss, 0, end, 0, False, 60, 3)
        assert_same(g, o)


def _rows(ts, vals):
    return I(list(zip(ts, vals)), minimal=False)


def test_same_bounds_other_cadence_reruns(ctx):
    """every span starts and ends at the same second, but one has a coarser
    cadence: its buckets differ, the group is rerun with E"""
    rng = np.random.default_rng(1)
    spans = [_rows(range(T0, T0 + 3599), rng.integers(-10**6, 10**6, 3599)) for _ in range(20)]
    spans.insert(7, _rows(range(T0, T0 + 3599, 2), rng.integers(-10**6, 10**6, 1800)))
    ss = packing.pack_spans(spans)
    for agg in (0, 1, 2, 3):
        g, o = run_both(ctx, ss, 0, U32MAX, agg, False, 60, 3)
        assert_same(g, o)
        assert paths(ctx) & _abi.PATH_ALIGNED_RERUN


def test_float_span_in_aligned_group_reruns(ctx):
    """a float series among aligned integer ones (double buckets: not
    combined out of order)"""
    rng = np.random.default_rng(2)
    spans = [_rows(range(T0, T0 + 1200), rng.integers(0, 1000, 1200)) for _ in range(10)]
    spans.append(F([(t, float(v)) for t, v in zip(range(T0, T0 + 1200), rng.standard_normal(1200))]))
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss, 0, U32MAX, 0, False, 60, 3)
    assert_same(g, o)
    assert paths(ctx) & _abi.PATH_ALIGNED_RERUN


def test_not_tried(ctx):
    """dev, rate, more than 64 buckets a span, spans of different bounds: the
    usual path"""
    ss = synth.regular(50, 3600, I64, seed=4, step=1)
    for kw in (dict(agg=4, dsa=3, dsi=60), dict(agg=0, dsa=4, dsi=60), dict(agg=0, dsa=3, dsi=30),
               dict(agg=0, dsa=3, dsi=60, rate=True)):
        g, o = run_both(ctx, ss, 0, U32MAX, kw["agg"], kw.get("rate", False), kw["dsi"], kw["dsa"])
        assert_same(g, o)
        assert not (paths(ctx) & (_abi.PATH_ALIGNED_GROUP | _abi.PATH_ALIGNED_RERUN))
    ss = synth.jittered(30, 200, seed=2, span_range=200_000, max_gap=60)
    g, o = run_both(ctx, ss, 0, U32MAX, 0, False, 60, 3)
    assert_same(g, o)


def test_exact_order(ctx):
    ss = synth.regular(200, 3600, I64, seed=8, step=1)
    g, o = run_both(ctx, ss, 0, U32MAX, 0, False, 60, 3, exact=True)
    assert_same(g, o)
    assert paths(ctx) & _abi.PATH_ALIGNED_GROUP


@pytest.fixture(scope="module", params=[2, 4])
def mctx(request):
    from opentsdb_amd._lib import Context
    c = Context(devices=[0] * request.param)
    yield c
    c.close()


@pytest.mark.parametrize("agg", [0, 1, 2, 3])
def test_aligned_group_sharded(mctx, agg):
    """each rank's shard is an aligned group whose grid is the global one;
    its partials enter the exchange as a 1-chunk reduce would"""
    import oracle
    ss = synth.regular(130, 3600, I64, seed=9, step=1)
    g = core.run_spanset(mctx, ss, 0, U32MAX, agg, False, 60, 3)
    o = oracle.spangroup(ss, 0, U32MAX, agg, False, 60, 3)
    assert_same(g, o)
    assert paths(mctx) & _abi.PATH_ALIGNED_GROUP
