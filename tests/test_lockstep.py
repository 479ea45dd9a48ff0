"""The lockstep path (k_direct_opt + k_lockstep, no downsampling): every kept
span one row on the same cadence (x0, n, step), width and type — C3's
shape. k_direct_opt proposes the group from three qualifiers a span;
k_lockstep proves every other qualifier while it streams the values, and a
proposal that does not hold makes the call run again on the proven path
(tsdbhip_timing.paths: PATH_LOCKSTEP / PATH_DIRECT_REDO). Every case is
checked against the oracle (SpanGroup.java:510-784, Aggregators.java:76-243):
integers bit-exact, doubles at 1e-9 relative; the corrupted-qualifier cases
check that the rerun reproduces the reference's results and errors."""
import numpy as np
import pytest

from helpers import I, F, T0, U32MAX, assert_same, corrupt_qual as corrupt, run_both, with_option
from opentsdb_amd import _abi, packing, synth

I64, F32, F64 = _abi.SYN_INT64_COUNTER, _abi.SYN_FLOAT32, _abi.SYN_FLOAT64
AGGS = [0, 1, 2, 3, 4]


@pytest.fixture(autouse=True)
def always(request):
    """these groups are small: "always" makes the proposal whatever the size
    ("on", the default, leaves groups of < 2048 lockstep waves to k_reduce)"""
    yield from with_option(request, "lockstep", "always", "on")


def tried(agg, rate):
    """the proposal is made unless the reduce is the span-ordered pass"""
    return agg != _abi.AGG_DEV or rate


def check_paths(ctx, lockstep, redo=False):
    p = ctx.timing().paths
    assert bool(p & _abi.PATH_LOCKSTEP) == lockstep, f"paths={p:#x}"
    assert bool(p & _abi.PATH_DIRECT_REDO) == redo, f"paths={p:#x}"


@pytest.mark.gpu
@pytest.mark.parametrize("kind", [I64, F32, F64])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_lockstep_regular(ctx, kind, agg, rate):
    ss = synth.regular(300, 1300, kind, seed=5, step=2)
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    check_paths(ctx, tried(agg, rate))


@pytest.mark.gpu
@pytest.mark.parametrize("n_points", [2, 3, 9, 511, 512, 513, 1024, 1025, 3600])
@pytest.mark.parametrize("rate", [False, True])
def test_lockstep_tile_edges(ctx, n_points, rate):
    """grids of one partial tile, exact multiples of the 512-point tile, one
    point past them (rate: the last cell is proven by k_direct_opt alone).
    Rows of fewer than 64 cells on average take the general decode, not the
    streaming (direct / lockstep) kernels."""
    ss = synth.regular(70, n_points, I64, seed=9, step=1)
    for agg in (0, 2):
        g, o = run_both(ctx, ss, agg=agg, rate=rate)
        assert_same(g, o)
        check_paths(ctx, n_points >= 64)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_lockstep_int32_and_many_chunks(ctx, agg, rate):
    """4-byte ints (minimal-width writes of values past 16 bits) over enough
    spans for dozens of span chunks, combined in chunk order"""
    spans = [I([(T0 + 3 * i, 1_000_000 + 7 * i * (s + 1) - 50_000 * (s % 3)) for i in range(600)]) for s in range(3000)]
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    check_paths(ctx, tried(agg, rate))


@pytest.mark.gpu
def test_lockstep_staggered_is_not_lockstep(ctx):
    """spans on one cadence but different phases: no single class key, the
    proven direct path runs (no rerun)"""
    spans = [I([(T0 + (s % 5) + 5 * i, s * 10 + i) for i in range(500)], minimal=False) for s in range(40)]
    ss = packing.pack_spans(spans)
    for rate in (False, True):
        g, o = run_both(ctx, ss, agg=0, rate=rate)
        assert_same(g, o)
        check_paths(ctx, False)


CORRUPTIONS = {
    "delta+1": lambda q: q + 16,                   # off the cadence, still increasing (step 2)
    "float-flag": lambda q: q | 0x8,               # an 8-byte double cell among longs
    "width-4": lambda q: (q & ~0x7) | 0x3,         # a 4-byte cell: later values misread
    "width-3": lambda q: (q & ~0x7) | 0x2,         # an illegal width: IllegalDataException
}


@pytest.mark.gpu
@pytest.mark.parametrize("what", sorted(CORRUPTIONS))
@pytest.mark.parametrize("cell", [100, 1100])
@pytest.mark.parametrize("rate", [False, True])
def test_lockstep_corrupt_middle_cell_reruns(ctx, what, cell, rate):
    """a qualifier the proposal never read (neither cell 0, 1 nor the last):
    k_lockstep sees it differ, the call runs again on the proven path and
    matches the reference, errors and their lazy index included"""
    ss = corrupt(synth.regular(200, 1300, I64, seed=3, step=2), 117, cell, CORRUPTIONS[what])
    for agg in (0, 2):
        g, o = run_both(ctx, ss, agg=agg, rate=rate)
        assert_same(g, o)
        check_paths(ctx, False, redo=True)


@pytest.mark.gpu
@pytest.mark.parametrize("cell", [0, 1, 1299])
def test_lockstep_corrupt_probed_cell(ctx, cell):
    """a qualifier k_direct_opt reads: the span proposes nothing, the group is
    not lockstep, the scan takes it (no rerun)"""
    ss = corrupt(synth.regular(200, 1300, I64, seed=3, step=2), 5, cell, CORRUPTIONS["delta+1"])
    g, o = run_both(ctx, ss, agg=0)
    assert_same(g, o)
    check_paths(ctx, False)


@pytest.mark.gpu
def test_lockstep_window(ctx):
    """start / end inside the spans: no proposal (points outside the window);
    the window exactly around them: lockstep"""
    ss = synth.regular(50, 1000, I64, seed=2, step=1)
    g, o = run_both(ctx, ss, start=T0 + 10, end=U32MAX, agg=0)
    assert_same(g, o)
    check_paths(ctx, False)
    g, o = run_both(ctx, ss, start=T0 + 10, end=T0 + 500, agg=0)
    assert_same(g, o)
    check_paths(ctx, False)
    g, o = run_both(ctx, ss, start=T0, end=T0 + 999, agg=0)
    assert_same(g, o)
    check_paths(ctx, True)


@pytest.mark.gpu
def test_lockstep_nan_result(ctx):
    """float spans whose aggregate is NaN at one t: IllegalStateException at
    that output index, from the lockstep reduce (no rerun)"""
    spans = [F([(T0 + i, 1.0 + i) for i in range(700)], double=True) for _ in range(5)]
    spans.append(F([(T0 + i, float("nan") if i == 600 else 2.0) for i in range(700)], double=True))
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss, agg=0)
    assert o.code == _abi.E_NAN_INF
    assert_same(g, o)
    check_paths(ctx, True)


@pytest.mark.gpu
def test_lockstep_auto_skips_small_groups(ctx):
    """the default ("on"): C1's shape (100 spans x 3600) takes k_reduce, no
    proposal; a group of >= 2048 lockstep waves takes k_lockstep"""
    ss = synth.regular(100, 3600, I64, seed=1, step=1)
    ctx.set_option("lockstep", "on")
    g, o = run_both(ctx, ss, agg=0)
    assert_same(g, o)
    check_paths(ctx, False)
    ss = synth.regular(20_000, 600, I64, seed=1, step=1)  # 2 tiles x 312 chunks of 64 spans
    g, o = run_both(ctx, ss, agg=0)
    assert_same(g, o)
    check_paths(ctx, False)
    ss = synth.regular(70_000, 600, I64, seed=1, step=1)  # 2 x 1093
    g, o = run_both(ctx, ss, agg=0)
    assert_same(g, o)
    check_paths(ctx, True)
