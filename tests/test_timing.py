"""tsdbhip_timing_totals: per-call HIP-event timings summed by the library
(what bench.py reads once after its timed loop), against the per-call
tsdbhip_last_timing readouts of the same calls."""
import pytest

from helpers import run_both, assert_same
from opentsdb_amd import core, synth, _abi

pytestmark = pytest.mark.gpu


def test_timing_totals_sum_the_calls(ctx):
    ss = synth.regular(50, 3600, _abi.SYN_INT64_COUNTER, seed=11, step=1)
    ctx.timing_totals(reset=True)
    per_call = []
    for _ in range(5):
        core.run_spanset(ctx, ss, 0, (1 << 32) - 1, 0, False, 60, 3)
        per_call.append(ctx.timing())
    tsum, n = ctx.timing_totals(reset=True)
    assert n == 5
    assert abs(tsum.total_ms - sum(t.total_ms for t in per_call)) <= 1e-3 * max(1.0, tsum.total_ms)
    assert abs(tsum.hot_ms - sum(t.hot_ms for t in per_call)) <= 1e-3 * max(1.0, tsum.hot_ms)
    assert tsum.n_grid == sum(int(t.n_grid) for t in per_call)
    assert tsum.hot_kernel == per_call[-1].hot_kernel
    _, n2 = ctx.timing_totals()
    assert n2 == 0  # (reset)


def test_calls_after_an_error_start_clean(ctx):
    """A call that throws mid-way (here E_EMPTY_SPAN at the first round trip)
    leaves its call state and grid bitmap dirty; the next calls on the context
    re-initialise them (no state carried over), for every path."""
    import numpy as np
    from helpers import I, T0
    from opentsdb_amd import packing
    good = synth.regular(20, 600, _abi.SYN_INT64_COUNTER, seed=3, step=1)
    bad = packing.pack_spans([I([(T0 + 1, 1), (T0 + 2, 2)])])
    bad.span_row_start = np.array([0, 1, 1], np.uint64)
    for dsi in (0, 60):
        g, o = run_both(ctx, good, agg=0, ds_interval=dsi, ds_agg=3)
        assert_same(g, o)
        gb, ob = run_both(ctx, bad, agg=0, ds_interval=dsi, ds_agg=3)
        assert gb[0] == ob.code == _abi.E_EMPTY_SPAN
        for _ in range(2):
            g, o = run_both(ctx, good, agg=0, ds_interval=dsi, ds_agg=3)
            assert_same(g, o)
