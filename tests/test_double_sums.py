"""The default (not EXACT_ORDER) double sum of the general reducer (ADVICE r3,
low): spans with no point in a 64-point tile contribute one line in t,
sum_s v_s(t_first) + (t - t_first) * sum_s slope_s (k_reduce.hip), instead of
the reference's per-span lerp-then-add (SpanGroup.java:736-784 with the
sequential Aggregators.SUM, Aggregators.java:76-104). That changes rounding
only; the error of each output is bounded by a few ulps of the sum of
|terms| at that t (each slope's rounding is scaled by t - t_first < 64
tile steps, not by t itself). These groups make the slopes large and of
opposite signs, so the sums cancel to a small fraction of sum |terms|, and
check the default order against the oracle at 1e-9 of sum |terms| (the
oracle's own aggregation over |values|: |lerp(v)| <= lerp(|v|)), and
EXACT_ORDER bit-exactly."""
import numpy as np
import pytest

import oracle
from helpers import F, I, T0, U32MAX, assert_same
from opentsdb_amd import _abi, core, packing


def groups(seed, absval=False):
    return packing.pack_spans(groups_list(seed, absval))


def groups_list(seed, absval=False):
    rng = np.random.default_rng(seed)
    spans = []
    for s in range(100):  # sparse double series: long brackets over many tiles
        off = int(rng.integers(0, 90_000))
        ts = [T0 + off + 100_000 * k for k in range(12)]
        vals = rng.uniform(-1e12, 1e12, len(ts)) * (1 if s % 2 else -1)
        if absval:
            vals = np.abs(vals)
        spans.append(F(list(zip(ts, vals.tolist())), double=True))
    # a dense integer series: grid points every 7 s, so the tiles of 64 points
    # lie inside the sparse series' brackets
    drv = [(T0 + 7 * i, (1000 + i) if absval else (1000 + i) * (1 if i % 3 else -1)) for i in range(150_000)]
    spans.append(I(drv, minimal=False))
    return spans


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("agg", [_abi.AGG_SUM, _abi.AGG_AVG])
def test_opposite_slopes_line_in_t(ctx, seed, agg):
    ss, sa = groups(seed), groups(seed, absval=True)
    o = oracle.spangroup(ss, 0, U32MAX, agg)
    oa = oracle.spangroup(sa, 0, U32MAX, agg)
    assert o.code == 0 and np.array_equal(o.ts, oa.ts) and len(o.ts) > 100_000
    scale = np.where(oa.is_int.astype(bool), oa.bits.astype(np.float64), oa.bits.view(np.float64))
    dbl = ~o.is_int.astype(bool)
    res = o.bits.view(np.float64)
    assert np.median(np.abs(res[dbl]) / scale[dbl]) < 0.5  # (the sums cancel)
    g = core.run_spanset(ctx, ss, 0, U32MAX, agg)
    assert_same(g, o, abs_scale=scale)
    # (registered result buffers: each tile group finalized by the reduce into them)
    g = core.run_spanset(ctx, ss, 0, U32MAX, agg, register_out=True)
    assert_same(g, o, abs_scale=scale)
    gx = core.run_spanset(ctx, ss, 0, U32MAX, agg, exact=True)
    assert_same(gx, o, exact_double=True)


@pytest.mark.gpu
@pytest.mark.parametrize("register_out", [False, True])
def test_nan_in_a_long_grid(ctx, register_out):
    """a NaN value mid-way through a long grid: IllegalStateException at the
    first NaN output (SpanGroup.java:660-663), also when the reduce finalizes
    into the caller's registered buffers"""
    spans = [F([(T0 + 7 * i + 3, float("nan") if i == 60_000 else 1.5) for i in range(100_000)], double=True)]
    base = groups_list(3) + spans
    ss = packing.pack_spans(base)
    o = oracle.spangroup(ss, 0, U32MAX, _abi.AGG_SUM)
    assert o.code == _abi.E_NAN_INF and o.err_index > 100_000
    g = core.run_spanset(ctx, ss, 0, U32MAX, _abi.AGG_SUM, register_out=register_out)
    assert g[0] != _abi.E_HIP, ctx.last_error()
    assert_same(g, o)
