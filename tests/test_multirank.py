"""N-rank series sharding on one GPU (the exchange had only ever
run on a 1-rank communicator). A context over devices [0] * N splits every
SpanGroup into N contiguous span ranges, one host thread per rank, and the
ranks exchange bounds, flags, grid bitmaps and per-t partials through the
same collectives the RCCL path issues (LocalXchg: device copies ordered by
HIP events); results are compared with the oracle on the whole group:
integers (integer dev included: the span-ordered pass continues from rank to
rank) bit-exact, doubles at 1e-9 relative, or bit-exact with EXACT_ORDER.
Shards get differing grids (jittered spans), mixed int/float, every
aggregator, ranks without spans, and errors raised inside a non-zero rank's
shard. The last test drives one context and per-thread contexts from 8 host
threads at once (re-entrancy)."""
import threading

import numpy as np
import pytest

import oracle
from helpers import I, F, T0, U32MAX, assert_same, corrupt_qual
from opentsdb_amd import _abi, core, packing, synth

AGGS = [0, 1, 2, 3, 4]


@pytest.fixture(scope="module", params=[2, 4, 8])
def mctx(request):
    from opentsdb_amd._lib import Context
    c = Context(devices=[0] * request.param)
    assert c.ranks == request.param
    yield c
    c.close()


def both(c, ss, start=0, end=U32MAX, agg=0, rate=False, dsi=0, dsa=0, exact=False):
    g = core.run_spanset(c, ss, start, end, agg, rate, dsi, dsa, exact=exact)
    o = oracle.spangroup(ss, start, end, agg, rate, dsi, dsa)
    return g, o


@pytest.mark.gpu
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_regular_downsampled(mctx, agg, rate):
    ss = synth.regular(40, 2000, _abi.SYN_INT64_COUNTER, seed=7, step=10)
    g, o = both(mctx, ss, agg=agg, rate=rate, dsi=60, dsa=3)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_regular_direct(mctx, agg, rate):
    """no downsampling: the direct path's consecutive-rank check against the
    exchanged grid"""
    ss = synth.regular(33, 1300, _abi.SYN_INT64_COUNTER, seed=5, step=5)
    g, o = both(mctx, ss, agg=agg, rate=rate)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", AGGS)
def test_c3s_shape_many_chunks(mctx, agg):
    """>= 64 reduce chunks per rank, their in-order combine before the exchange"""
    ss = synth.regular(2100, 600, _abi.SYN_INT64_COUNTER, seed=11, step=1)
    g, o = both(mctx, ss, agg=agg, dsi=60, dsa=3)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_jittered_mixed_differing_grids(mctx, seed, agg, rate):
    """each shard's grid differs (allgather + OR of the bitmaps); mixed
    int/float series, so the double path and F* travel between ranks"""
    ss = synth.jittered(13, 70, seed=seed, span_range=400_000, max_gap=700)
    g, o = both(mctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    g, o = both(mctx, ss, agg=agg, rate=rate, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [4, 5, 6])
@pytest.mark.parametrize("agg", AGGS)
def test_jittered_int_lerp(mctx, seed, agg):
    """all-integer jittered series: int64 lerp; integer dev bit-exact"""
    ss = synth.jittered(17, 90, seed=seed, span_range=300_000, max_gap=900, float_frac=0.0, float_cell_frac=0.0)
    g, o = both(mctx, ss, agg=agg)
    assert_same(g, o, exact_double=True)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 3, 4])
def test_integer_dev_large_values(mctx, agg):
    """dev over 8-byte counters near 2^40 (C3's values): Chan merges of
    shard states would differ from the sequential Welford in the last bits,
    which the (long) cast exposes"""
    ss = synth.regular(300, 700, _abi.SYN_INT64_COUNTER, seed=3, step=1)
    g, o = both(mctx, ss, agg=agg)
    assert_same(g, o, exact_double=True)


@pytest.mark.gpu
def test_fewer_spans_than_ranks(mctx):
    ss = packing.pack_spans([I([(T0 + 10 * i, i) for i in range(40)]), F([(T0 + 5 + 7 * i, 0.5 * i) for i in range(30)])])
    for agg in AGGS:
        g, o = both(mctx, ss, agg=agg)
        assert_same(g, o)
    ss = packing.pack_spans([])
    g, o = both(mctx, ss)
    assert_same(g, o)


@pytest.mark.gpu
def test_illegal_cell_in_a_later_rank(mctx):
    """the IllegalDataException's lazy index comes from the rank holding the
    bad cell (allreduced), every rank agrees on the code"""
    T = T0
    bad = packing.KeyValue(T, bytes([0x00, 0x02, 0x00, 0x12]), bytes([1, 2, 3, 4, 5, 6, 0]))  # 3-byte ints
    spans = [I([(T + i, i) for i in range(5)]) for _ in range(5)] + [[bad]]
    ss = packing.pack_spans(spans)
    g, o = both(mctx, ss)
    assert g[0] == _abi.E_ILLEGAL_DATA
    assert_same(g, o)


@pytest.mark.gpu
def test_empty_span_and_nan_in_a_later_rank(mctx):
    T = T0
    ss = packing.pack_spans([I([(T + 1, 1), (T + 2, 2)])] * 6)
    ss.span_row_start = np.concatenate([ss.span_row_start, [ss.span_row_start[-1]]]).astype(np.uint64)
    g, o = both(mctx, ss)
    assert o.code == _abi.E_EMPTY_SPAN
    assert_same(g, o)
    spans = [F([(T + 1, 1.0), (T + 2, 1.0)])] * 5 + [F([(T + 1, float("inf")), (T + 2, 1.0)])]
    g, o = both(mctx, packing.pack_spans(spans))
    assert g[0] == _abi.E_NAN_INF
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("dsi", [60, 0])
def test_aligned_grids_skip_the_grid_exchange(mctx, dsi):
    """Aligned shards (C3* / C3: every series on the same cadence): each
    rank's local grid is the global one, which the agreement header proves,
    so a call issues two collective launches, the header and the partials
     -- one when downsampled: the aligned group's partials
    travel in the header's collective group. Without downsampling these
    shards take the uniform lockstep path: the key agreement, then the
    partials. Shards whose grids differ also exchange bitmaps (after the
    uniform path's key agreement, which every rank issues for such a query)."""
    ss = synth.regular(64, 600, _abi.SYN_INT64_COUNTER, seed=2, step=1)
    for agg in (0, 2):
        g, o = both(mctx, ss, agg=agg, dsi=dsi, dsa=3)
        assert_same(g, o)
        assert mctx.timing().n_collectives == (1 if dsi else 2)
    ss = synth.jittered(13, 70, seed=1, span_range=400_000, max_gap=700)
    g, o = both(mctx, ss, agg=0)
    assert_same(g, o)
    assert mctx.timing().n_collectives == 4


@pytest.mark.gpu
@pytest.mark.timeout(120)
@pytest.mark.parametrize("agg", [0, 2, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_equal_bucket_grids_different_last_ts(mctx, agg, rate):
    """shards whose bucket grids are equal while their raw
    [first, last] ranges differ (the first half of the spans end one second
    later than the second half). Each rank's bitmap and hashes match, only hi
    differs, so a decision that compared a rank's own hi with the agreed max
    split the ranks (the one holding the max took the agreed branch, its
    peers the allgather: a deadlock). The decision now reads the agreed words
    alone. Covers the aligned-group finish (sum / max) and the usual path
    (dev, rate)."""
    n = 2 * mctx.ranks
    length = 120
    spans = [I([(T0 + i, 1000 * s + i) for i in range(length - (s >= n // 2))]) for s in range(n)]
    ss = packing.pack_spans(spans)
    g, o = both(mctx, ss, agg=agg, rate=rate, dsi=60, dsa=3)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 2, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_lockstep_sharded(mctx, agg, rate):
    """every rank's shard lockstep on the same cadence (C3's shape): each rank
    reduces its spans with k_lockstep, the partials travel as usual"""
    ss = synth.regular(64, 900, _abi.SYN_INT64_COUNTER, seed=4, step=1)
    g, o = both(mctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    p = mctx.timing().paths
    assert bool(p & _abi.PATH_LOCKSTEP) == (agg != 4 or rate) and not p & _abi.PATH_DIRECT_REDO


@pytest.mark.gpu
@pytest.mark.parametrize("rate", [False, True])
def test_lockstep_sharded_broken_in_last_rank(mctx, rate):
    """a qualifier off the cadence in the last rank's shard: that rank's
    k_lockstep flags it, the flag is agreed in the partials' collective group
    and every rank runs the call again on the proven path"""
    ss = corrupt_qual(synth.regular(64, 900, _abi.SYN_INT64_COUNTER, seed=4, step=2), 63, 400, lambda q: q + 16)
    g, o = both(mctx, ss, agg=0, rate=rate)
    assert_same(g, o)
    p = mctx.timing().paths
    assert p & _abi.PATH_DIRECT_REDO and not p & _abi.PATH_LOCKSTEP


@pytest.mark.gpu
def test_lockstep_sharded_ranks_disagree(mctx):
    """each rank lockstep on its own, but on different phases: the global
    grid is wider than every rank's pattern, so no rank may use its proposal
    (unproven spans): broken everywhere, rerun"""
    n = 4 * mctx.ranks
    spans = [I([(T0 + (s >= n // 2) + 2 * i, s * 7 + i) for i in range(800)], minimal=False) for s in range(n)]
    ss = packing.pack_spans(spans)
    for agg, rate in ((0, False), (2, True)):
        g, o = both(mctx, ss, agg=agg, rate=rate)
        assert_same(g, o)
        assert mctx.timing().paths & _abi.PATH_DIRECT_REDO


@pytest.mark.gpu
@pytest.mark.timeout(120)
@pytest.mark.parametrize("rate", [False, True])
def test_lockstep_broken_next_to_an_empty_rank(mctx, rate):
    """fewer spans than ranks, one qualifier off the cadence.
    The ranks holding spans try the lockstep proposal and break it; the empty
    rank never tries. The rerun is decided from the agreed flag alone, so the
    empty rank reruns too (a per-rank decision left its peers waiting in the
    rerun's collectives)."""
    n = mctx.ranks - 1
    ss = synth.regular(n, 900, _abi.SYN_INT64_COUNTER, seed=4, step=2)
    ss = corrupt_qual(ss, n - 1, 400, lambda q: q + 16)
    for agg in (0, 2):
        g, o = both(mctx, ss, agg=agg, rate=rate)
        assert_same(g, o)
        assert mctx.timing().paths & _abi.PATH_DIRECT_REDO


@pytest.mark.gpu
@pytest.mark.timeout(120)
def test_lockstep_broken_next_to_a_short_row_rank(mctx):
    """the last rank's shard is a series of short rows (the
    general decode: no lockstep try there) while the other ranks' proposal is
    broken by a corrupted qualifier: every rank reruns"""
    n = mctx.ranks - 1
    spans = [I([(T0 + 2 * i, 1000 * s + 3 * i) for i in range(900)], minimal=False) for s in range(n)]
    # 20 points on the same grid in one row: < 64 cells a row, the general decode
    sparse = I([(T0 + 2 * i, i) for i in range(0, 900, 45)], minimal=False)
    ss = corrupt_qual(packing.pack_spans(spans + [sparse]), 0, 300, lambda q: q + 16)
    for agg, rate in ((0, False), (2, True)):
        g, o = both(mctx, ss, agg=agg, rate=rate)
        assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.timeout(120)
@pytest.mark.parametrize("agg", [0, 1, 3])
def test_lockstep_int_shard_next_to_float_shard(mctx, agg):
    """int shards and float shards on one cadence. Each rank
    proposes lockstep in its own cell type, but the group's reduce mode is the
    agreed dual one: an int rank's MODE_INT partials would leave the double
    fields unwritten. Such a rank cannot use its proposal: every rank reruns
    on the proven path."""
    n = 2 * mctx.ranks
    spans = [I([(T0 + 2 * i, 100 * s + i) for i in range(700)], minimal=False) for s in range(n // 2)]
    spans += [F([(T0 + 2 * i, 0.5 * s + i) for i in range(700)], double=True) for s in range(n // 2)]
    ss = packing.pack_spans(spans)
    g, o = both(mctx, ss, agg=agg)
    assert_same(g, o)
    assert mctx.timing().paths & _abi.PATH_DIRECT_REDO


@pytest.mark.gpu
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_long_grid_sliced_exchange(mctx, agg, rate):
    """a union grid of > 64k points with double partials
    (mixed int/float jittered series): each rank owns 1/N of G, receives the
    ranks' partials of its slice only (alltoall), merges them in rank order
    (SpanGroup.java:647-667) and finalizes it; the slices' results are
    gathered. Compared with the whole-group oracle; the sum case also checks
    the bytes a rank received: (N-1)/N of its 21-B dual-mode partials plus the
    17-B results, instead of N-1 times all of them (from 3 ranks on)."""
    ss = synth.jittered(60, 2000, seed=8, span_range=3_000_000, max_gap=3000)
    g, o = both(mctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    T, N = len(o.ts), mctx.ranks
    assert T >= 65536
    if agg == 0 and not rate:
        bitmap = (N - 1) * ((int(ss.row_base.max()) + 3600 - int(ss.row_base.min())) // 32 + 2) * 4
        x = mctx.timing().x_bytes
        if N == 2:  # (no gain from slices at 2 ranks: every partial gathered)
            assert (N - 1) * T * 21 <= x <= (N - 1) * T * 21 + bitmap + 4096, (x, T, bitmap)
        else:
            xs = (T + N - 1) // N
            lo_x = (N - 1) * xs * (21 + 17)
            assert lo_x <= x <= lo_x + bitmap + 4096, (x, lo_x, bitmap)


@pytest.mark.gpu
def test_error_order_is_global_span_order(mctx, ctx):
    """Two Span.addRow errors at the same base time in different ranks: the
    one in the lower global span wins (the scan's row-key order: base time,
    then span), whatever its index inside its own shard. Span 1
    (rank 0, local index 1) holds a row that goes back in time (-1, the
    IllegalDataException of Span.java:117-121), span 2 (rank 1, local index 0)
    an empty row at the same base (-9). Rows out of base order are outside the
    header's contract, so the expectation is the unsharded call's code."""
    T = T0
    n = 2 * mctx.ranks  # 10 cells per span: rank r holds spans 2r and 2r + 1
    spans = [I([(T + 3600 + i, i) for i in range(10)]) for _ in range(n)]
    spans[1] = I([(T + 3600 + i, i) for i in range(5)]) + I([(T + 100 + i, i) for i in range(5)])
    spans[2] = [packing.KeyValue(T, b"", b"")] + I([(T + 3600 + i, i) for i in range(10)])
    ss = packing.pack_spans(spans)
    whole = core.run_spanset(ctx, ss, 0, U32MAX, 0)
    assert whole[0] == _abi.E_ILLEGAL_DATA
    g = core.run_spanset(mctx, ss, 0, U32MAX, 0)
    assert g[0] == whole[0]


@pytest.mark.gpu
def test_error_stages_across_ranks_vs_oracle(mctx):
    """Errors in different ranks and stages, against the oracle:
    the reference throws the first it meets -- Span.addRow while the rows
    are scanned (an empty KeyValue: ArrayIndexOutOfBounds), then SpanGroup
    construction (an empty span: AssertionError, SpanGroup.java:452-455),
    then the lazy iteration (an illegal cell width, RowSeq.java:203, at its
    output index) -- whichever rank holds each. Rows sorted within spans (the
    header's contract)."""
    n = 3 * mctx.ranks
    good = lambda s: I([(T0 + 5 * i, 100 * s + i) for i in range(40)])  # noqa: E731
    bad_cell = packing.KeyValue(T0 + 3600, bytes([0x00, 0x02, 0x00, 0x12]), bytes([1, 2, 3, 4, 5, 6, 0]))
    spans = [good(s) for s in range(n)]
    spans[0] = spans[0] + [bad_cell]                       # lazy, rank 0
    spans[n - 1] = [packing.KeyValue(T0, b"", b"")] + spans[n - 1]  # scan, last rank
    for drop_scan in (False, True):
        sp = list(spans)
        if drop_scan:
            sp[n - 1] = good(n - 1)
        ss = packing.pack_spans(sp)
        # an empty span in rank 0 (SpanGroup construction)
        ss.span_row_start = np.concatenate([ss.span_row_start[:2], ss.span_row_start[1:]]).astype(np.uint64)
        g, o = both(mctx, ss)
        assert o.code == (_abi.E_EMPTY_SPAN if drop_scan else _abi.E_OUT_OF_BOUNDS)
        assert_same(g, o)
    ss = packing.pack_spans([good(s) for s in range(n - 1)] + [spans[0]])  # the bad cell in the last rank only
    g, o = both(mctx, ss)
    assert o.code == _abi.E_ILLEGAL_DATA and o.err_index > 0
    assert_same(g, o)


@pytest.mark.gpu
def test_device_desc_sharded(mctx):
    """device-resident input (tsdbhip_synth_generate) split by span count"""
    import ctypes as C
    d = _abi.SgDesc()
    p = _abi.SynthParams(seed=9, n_spans=150, n_points=900, t0=synth.T0, step=1, kind=_abi.SYN_INT64_COUNTER,
                         span0=0)
    mctx.check(mctx._lib.tsdbhip_synth_generate(mctx.handle, C.byref(p), C.byref(d)))
    try:
        ss = synth.regular(150, 900, _abi.SYN_INT64_COUNTER, seed=9, step=1)
        for agg, dsi in ((0, 60), (4, 0), (2, 0)):
            g = core.run_spanset(mctx, ss, 0, U32MAX, agg, False, dsi, 3 if dsi else 0, device_desc=d)
            o = oracle.spangroup(ss, 0, U32MAX, agg, False, dsi, 3 if dsi else 0)
            assert_same(g, o, exact_double=True)
    finally:
        mctx._lib.tsdbhip_synth_free(mctx.handle, C.byref(d))


# ------------------------------------------------------------ re-entrancy ----
def _workload(seed):
    rng = np.random.default_rng(seed)
    kind = int(rng.integers(0, 3))
    if kind == 0:
        ss = synth.regular(int(rng.integers(5, 60)), int(rng.integers(200, 3000)), _abi.SYN_INT64_COUNTER,
                           seed=seed, step=1)
        return ss, dict(agg=int(rng.integers(0, 5)), dsi=int(rng.choice([0, 60])), dsa=3, rate=bool(seed % 2))
    if kind == 1:
        ss = synth.jittered(int(rng.integers(3, 15)), 60, seed=seed, span_range=300_000, max_gap=900)
        return ss, dict(agg=int(rng.integers(0, 5)), dsi=0, dsa=0, rate=bool(seed % 3 == 0))
    ss = synth.regular(int(rng.integers(5, 40)), 1440, _abi.SYN_FLOAT32, seed=seed, step=10)
    return ss, dict(agg=3, dsi=60, dsa=3, rate=False)


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_concurrent_calls_shared_and_private_contexts(ctx):
    """8 host threads x 6 SpanGroups each, half on one shared context (one
    slot per concurrent call), half on a context of their own; every result
    checked against the oracle, and each thread's last_error / last_timing
    are its own."""
    from opentsdb_amd._lib import Context
    work = [[_workload(1000 * t + i) for i in range(6)] for t in range(8)]
    expected = [[oracle.spangroup(ss, 0, U32MAX, kw["agg"], kw["rate"], kw["dsi"], kw["dsa"]) for ss, kw in w]
                for w in work]
    errors = []
    barrier = threading.Barrier(8)

    def worker(t):
        try:
            c = ctx if t % 2 == 0 else Context(0)
            barrier.wait()
            for (ss, kw), o in zip(work[t], expected[t]):
                g = core.run_spanset(c, ss, 0, U32MAX, kw["agg"], kw["rate"], kw["dsi"], kw["dsa"])
                assert_same(g, o)
                assert c.timing().total_ms > 0
            # a failing call reports its own message on this thread
            bad = packing.pack_spans([I([(T0 + 1, 1)])])
            bad.span_row_start = np.array([0, 1, 1], np.uint64)
            assert core.run_spanset(c, bad, 0, U32MAX, 0)[0] == _abi.E_EMPTY_SPAN
            assert "error -3" in c.last_error()
            if c is not ctx:
                c.close()
        except Exception as e:  # reported below
            errors.append((t, repr(e)))

    th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    assert not errors, errors
