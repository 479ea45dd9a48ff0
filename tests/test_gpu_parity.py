"""GPU parity: libtsdbhip (HIP kernels, called through the C-ABI) vs the CPU
oracle (restatement of the reference, pinned by tests/golden) on the same
seeded inputs. Integer results are bit-exact; double results within 1e-9
relative, and bit-exact with TSDBHIP_EXACT_ORDER (one span chunk, the
reference's summation order)."""
import numpy as np
import pytest

from helpers import with_option, I, F, M, T0, U32MAX, run_both, assert_same
from opentsdb_amd import _abi, core, packing, synth

pytestmark = pytest.mark.gpu

AGGS = [0, 1, 2, 3, 4]


@pytest.fixture(autouse=True, params=["auto", "general", "fast", "chunks", "spans", "direct"])
def decode_path(request):
    """Run every case through the streaming downsamplers (chunks: the
    constant-step k_ds_reg first, then the chain-proved k_ds_spans; spans:
    k_ds_spans alone), the streaming decode kernel (each with its fallback
    queue), the general per-span kernel, and (no downsampling) the direct
    path of k_direct.hip forced on whatever the row sizes."""
    yield from with_option(request, "decode", request.param, "auto")


def ka_groups():
    T = T0
    return {
        "KA1": [I([(T + 100, 10), (T + 110, 20)]), I([(T + 105, 100), (T + 115, 200)])],
        "KA2": [I([(T + 100, 0), (T + 103, -10)]), I([(T + 101, 5)])],
        "KA3": [I([(T + 100, 10), (T + 110, 30), (T + 120, 60)]), I([(T + 105, 1000), (T + 115, 1100)])],
        "KA6": [I([(T + 100, 1), (T + 110, 2)]), F([(T + 200, 1.5), (T + 210, 2.5)])],
    }


@pytest.mark.parametrize("name", ["KA1", "KA2", "KA3", "KA6"])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_known_answers(ctx, name, agg, rate):
    ss = packing.pack_spans(ka_groups()[name])
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    g2, _ = run_both(ctx, ss, agg=agg, rate=rate, exact=True)
    assert_same(g2, o, exact_double=True)


def test_ka8_bracket_after_end(ctx):
    T = T0
    ss = packing.pack_spans([I([(T + 100, 0), (T + 200, 100)]), I([(T + 150, 7)])])
    g, o = run_both(ctx, ss, end=T + 160)
    assert_same(g, o, exact_double=True)
    assert list(g[1] - T) == [100, 150] and list(g[3]) == [0, 57]


@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("ds_agg", AGGS)
def test_downsample_ka4_ka5(ctx, agg, ds_agg):
    T = T0
    spans = [I([(T + 100 + i, i) for i in range(120)]),
             I([(T + 100, 1), (T + 130, 2), (T + 161, 3), (T + 170, 4), (T + 230, 5)])]
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss, agg=agg, ds_interval=60, ds_agg=ds_agg)
    assert_same(g, o)
    g, o = run_both(ctx, ss, agg=agg, ds_interval=60, ds_agg=ds_agg, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("kind", [_abi.SYN_INT64_COUNTER, _abi.SYN_FLOAT32, _abi.SYN_FLOAT64])
@pytest.mark.parametrize("agg", AGGS)
def test_regular_nods(ctx, kind, agg):
    ss = synth.regular(40, 700, kind, seed=3, step=10)
    g, o = run_both(ctx, ss, agg=agg)
    assert_same(g, o)
    g, o = run_both(ctx, ss, agg=agg, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("kind", [_abi.SYN_INT64_COUNTER, _abi.SYN_FLOAT32])
@pytest.mark.parametrize("agg,ds_agg", [(0, 3), (3, 3), (0, 0), (2, 1), (1, 2), (4, 4), (3, 4)])
@pytest.mark.parametrize("rate", [False, True])
def test_regular_ds(ctx, kind, agg, ds_agg, rate):
    ss = synth.regular(30, 2000, kind, seed=5, step=10)
    g, o = run_both(ctx, ss, agg=agg, rate=rate, ds_interval=60, ds_agg=ds_agg)
    assert_same(g, o)
    g, o = run_both(ctx, ss, agg=agg, rate=rate, ds_interval=60, ds_agg=ds_agg, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("seed", [1, 2, 3])
@pytest.mark.parametrize("agg", AGGS)
@pytest.mark.parametrize("rate", [False, True])
def test_jittered_mixed(ctx, seed, agg, rate):
    ss = synth.jittered(12, 60, seed=seed, span_range=400_000, max_gap=700)
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    g, o = run_both(ctx, ss, agg=agg, rate=rate, exact=True)
    assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("seed", [4, 5])
@pytest.mark.parametrize("agg", AGGS)
def test_jittered_int_lerp(ctx, seed, agg):
    """C4-int: all-integer series exercise the bit-exact int64 lerp."""
    ss = synth.jittered(15, 80, seed=seed, span_range=300_000, max_gap=900, float_frac=0.0,
                        float_cell_frac=0.0)
    g, o = run_both(ctx, ss, agg=agg)
    assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("seed", [6, 7])
@pytest.mark.parametrize("ds", [(300, 0), (300, 3), (900, 4), (120, 1)])
def test_jittered_ds(ctx, seed, ds):
    ss = synth.jittered(10, 80, seed=seed, span_range=200_000, max_gap=400)
    for agg in AGGS:
        g, o = run_both(ctx, ss, agg=agg, ds_interval=ds[0], ds_agg=ds[1], exact=True)
        assert_same(g, o, exact_double=True)


def regular_int_spans(n_spans, n_pts, step, seed, wide=True, perturb=None, offset_step=7):
    """Regular-cadence integer series, 8-byte cells (wide) or 4-byte ints;
    `perturb(s, ts_list)` may drop / shift points to break the cadence."""
    rng = np.random.default_rng(seed)
    spans = []
    for s in range(n_spans):
        ts = [T0 + 3 + s * offset_step + step * i for i in range(n_pts)]
        if perturb:
            ts = perturb(s, ts)
        if wide:
            vals = [int(v) for v in rng.integers(-(1 << 40), 1 << 40, len(ts))]
            spans.append(I(list(zip(ts, vals)), minimal=False))
        else:
            vals = [int(v) for v in rng.integers(1 << 17, 1 << 30, len(ts)) * rng.choice([-1, 1], len(ts))]
            spans.append(I(list(zip(ts, vals)), minimal=True))
    return packing.pack_spans(spans)


@pytest.mark.parametrize("step,interval", [(1, 60), (1, 45), (10, 60), (1, 7), (1, 1000), (2, 5000),
                                           (1, 1), (3, 2), (1, 100000)])
@pytest.mark.parametrize("ds_agg", [0, 1, 2, 3])
def test_chunk_regular(ctx, step, interval, ds_agg):
    """Chunk-parallel downsampling: buckets inside a chunk, spilling over
    chunks and hour rows, longer than a row, one cell per bucket, and a
    single bucket for the whole span."""
    ss = regular_int_spans(6, 3000, step, seed=interval + ds_agg)
    for agg in (0, 3, 1):
        g, o = run_both(ctx, ss, agg=agg, ds_interval=interval, ds_agg=ds_agg)
        assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("ds_agg", [0, 1, 2, 3])
def test_chunk_regular_int32_rows(ctx, ds_agg):
    ss = regular_int_spans(5, 2500, 1, seed=11, wide=False)
    g, o = run_both(ctx, ss, agg=0, ds_interval=60, ds_agg=ds_agg)
    assert_same(g, o, exact_double=True)


def _drop_one(s, ts):
    return ts[:700 + 97 * s] + ts[701 + 97 * s:]


def _shift_one(s, ts):
    out = list(ts)
    i = 1000 + 31 * s
    out[i] = out[i] - 1 if out[i] - 1 > out[i - 1] else out[i]
    return out


def _gap(s, ts):
    return ts[:500] + [t + 37 for t in ts[500:]] if s % 2 else ts


@pytest.mark.parametrize("perturb", [_drop_one, _shift_one, _gap])
@pytest.mark.parametrize("ds_agg", [0, 1, 2, 3])
def test_chunk_cadence_breaks(ctx, perturb, ds_agg):
    """A missing, shifted or gapped point breaks the regular-head hypothesis:
    the span must fall back to the serial kernels with identical results."""
    ss = regular_int_spans(8, 3000, 1, seed=21, perturb=perturb)
    for interval in (60, 13):
        g, o = run_both(ctx, ss, agg=0, ds_interval=interval, ds_agg=ds_agg)
        assert_same(g, o, exact_double=True)


def test_chunk_mixed_eligibility(ctx):
    """Regular wide int spans next to float, minimal-width, sparse and
    seek-start spans in one group."""
    T = T0
    spans = [I([(T + 3 + s * 7 + i, (i * 7919 + s) << 20) for i in range(2000)], minimal=False)
             for s in range(4)]
    spans += [F([(T + 3 + 2 * i, 0.25 * i) for i in range(1500)]),
              I([(T + 11 * i, i % 300) for i in range(400)]),
              I([(T + 500 + 997 * i, 5 * i) for i in range(6)])]
    ss = packing.pack_spans(spans)
    for ds_agg in (0, 1, 2, 3):
        for start in (0, T + 700):
            g, o = run_both(ctx, ss, start=start, agg=0, ds_interval=60, ds_agg=ds_agg)
            assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("window", [(100, 2000), (500, 1500), (0, 700), (1700, U32MAX)])
def test_start_end_windows(ctx, window):
    """start inside the data (seek), end cutting spans (brackets past end)."""
    T = T0
    spans = [I([(T + 10 * i, i * 7) for i in range(200)]),
             I([(T + 5 + 13 * i, -3 * i) for i in range(150)]),
             F([(T + 300 + 11 * i, 0.5 * i) for i in range(100)])]
    ss = packing.pack_spans(spans)
    lo, hi = window
    for agg in AGGS:
        for rate in (False, True):
            g, o = run_both(ctx, ss, start=T + lo, end=min(U32MAX, T + hi), agg=agg, rate=rate, exact=True)
            assert_same(g, o, exact_double=True)


def test_q1_seek_inside_row_minimal_widths(ctx):
    """Quirk Q1: a seek inside a row with non-1-byte values shifts offsets."""
    T = T0
    spans = [I([(T + i, 1000 + i) for i in range(50)], minimal=True),
             I([(T + i, 10 ** 6 + i) for i in range(50)], minimal=False)]
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        g, o = run_both(ctx, ss, start=T + 20, agg=agg, exact=True)
        assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("start_off", [3200, 3560, 3700, 3890])
def test_q1_seek_across_merged_rows(ctx, start_off):
    """Quirk Q1 where the RowSeq the seek lands in holds two merged hourly rows
    (the second row ends less than 4096 s after the first row's base,
    RowSeq.java:92-172): every later cell of the RowSeq is read at its offset
    in the merged values array minus the shift, so reads straddle the rows
    and, for a seek inside the second row, start in the first row's bytes."""
    T = T0
    rng = np.random.default_rng(start_off)
    mags = [0, 7, 15, 31, 40, 62]

    def vals(n):
        return [int(rng.integers(-(1 << 62), 1 << 62)) >> int(rng.choice(mags)) for _ in range(n)]

    pts_a = [T + 3000 + 7 * i for i in range(80)] + [T + 3600 + 5 * i for i in range(60)] + \
        [T + 7200 + 11 * i for i in range(30)]
    pts_b = [T + 3100 + 9 * i for i in range(50)] + [T + 3601 + 3 * i for i in range(90)]
    spans = [I(list(zip(pts_a, vals(len(pts_a)))), minimal=True),
             I(list(zip(pts_b, vals(len(pts_b)))), minimal=True),
             I([(T + 2900 + 13 * i, 5 * i) for i in range(100)], minimal=False)]
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        g, o = run_both(ctx, ss, start=T + start_off, agg=agg, exact=True)
        assert_same(g, o, exact_double=True)
    for dsi, dsa in ((60, 0), (45, 2)):
        g, o = run_both(ctx, ss, start=T + start_off, agg=0, ds_interval=dsi, ds_agg=dsa, exact=True)
        assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("seed", [21, 22])
def test_cached_long_lerp_bounds(ctx, seed):
    """Long lerp of a span with no point in a tile (the cached bracket):
    |y1 - y0| just under, at and over 2^31 - 1 (the double-estimate quotient
    vs the general 64-bit division), both signs, quotients that land exactly
    on integers, and brackets up to 2^24 s wide under a dense span."""
    T = T0
    rng = np.random.default_rng(seed)
    dense = I([(T + 1 + 3 * i, int(v)) for i, v in enumerate(rng.integers(-9, 9, 3000))], minimal=True)
    spans = [dense]
    M31 = (1 << 31) - 1
    for dy in (M31 - 2, M31 - 1, M31, M31 + 1, 1 << 40, 8999, 9000, 1):
        for sign in (1, -1):
            y0 = int(rng.integers(-(1 << 50), 1 << 50))
            d = int(rng.choice([9000, 7, 4096, 1 << 24]))
            x0 = T + int(rng.integers(0, 40))
            spans.append(I([(x0, y0), (x0 + d, y0 + sign * dy), (x0 + d + 5, y0)], minimal=True))
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        g, o = run_both(ctx, ss, agg=agg, exact=True)
        assert_same(g, o, exact_double=True)
        g, o = run_both(ctx, ss, agg=agg)
        assert_same(g, o)


def test_minimal_width_ints(ctx):
    T = T0
    rng = np.random.default_rng(9)
    spans = []
    for s in range(6):
        vals = rng.integers(-(1 << 40), 1 << 40, 300) >> rng.integers(0, 40, 300)
        spans.append(I([(T + 3 * i + s, int(v)) for i, v in enumerate(vals)], minimal=True))
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        g, o = run_both(ctx, ss, agg=agg)
        assert_same(g, o, exact_double=True)


def test_empty_and_disjoint(ctx):
    T = T0
    ss = packing.pack_spans([I([(T + 100, 1)])])
    g, o = run_both(ctx, ss, start=T + 200, end=T + 300)
    assert_same(g, o)
    assert len(g[1]) == 0
    ss = packing.pack_spans([])
    g, o = run_both(ctx, ss)
    assert_same(g, o)
    # a span without rows: Span.timestamp(0) throws in SpanGroup.add
    ss = packing.pack_spans([I([(T + 1, 1), (T + 2, 2)])])
    ss.span_row_start = np.array([0, 1, 1], np.uint64)
    g, o = run_both(ctx, ss)
    assert o.code == _abi.E_EMPTY_SPAN
    assert_same(g, o)


def test_error_priority_scan_before_group(ctx):
    """Two errors: an empty span (thrown by SpanGroup.add) ahead of a row that
    Span.addRow rejects in a later span. The scanner's addRow calls all run
    before the group is built (TsdbQuery.java:240-307), so the later span's
    error wins."""
    T = T0
    bad = packing.KeyValue(T + 3600, b"", b"")
    for spans in ([I([(T + 1, 1), (T + 2, 2)]), [], I([(T + 5, 3)]) + [bad]],
                  [I([(T + 1, 1)]), [], [bad]]):
        ss = packing.pack_spans(spans)
        g, o = run_both(ctx, ss)
        assert o.code == _abi.E_OUT_OF_BOUNDS
        assert_same(g, o)


def test_single_point_rate(ctx):
    T = T0
    ss = packing.pack_spans([I([(T + 100, 5)]), I([(T + 50, 1), (T + 150, 9)])])
    for agg in AGGS:
        g, o = run_both(ctx, ss, agg=agg, rate=True)
        assert_same(g, o, exact_double=True)


def test_illegal_width(ctx):
    T = T0
    bad = packing.KeyValue(T, bytes([0x00, 0x02, 0x00, 0x12]), bytes([1, 2, 3, 4, 5, 6, 0]))  # len 3 ints
    spans = [I([(T + i, i) for i in range(5)]), [bad]]
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss)
    assert_same(g, o)
    assert g[0] == _abi.E_ILLEGAL_DATA


def test_nan_result(ctx):
    T = T0
    spans = [F([(T + 1, float("inf")), (T + 2, 1.0)]), F([(T + 1, 1.0), (T + 2, 1.0)])]
    ss = packing.pack_spans(spans)
    g, o = run_both(ctx, ss)
    assert_same(g, o)
    assert g[0] == _abi.E_NAN_INF


def test_row_assembly_rules(ctx):
    """Span.addRow: out-of-order rows dropped, merges of close rows."""
    T = T0
    r1 = synth.compact_cells(T, [(T + i, 0x7, int(i).to_bytes(8, "big")) for i in range(0, 3600, 7)])
    r2 = synth.compact_cells(T + 3600, [(T + 3600 + i, 0x7, int(i).to_bytes(8, "big")) for i in range(0, 400, 3)])
    r_old = synth.compact_cells(T, [(T + 5, 0x0, bytes([9]))])
    r3 = synth.compact_cells(T + 7200, [(T + 7200 + i, 0x3, int(i).to_bytes(4, "big")) for i in range(0, 3600, 11)])
    spans = [[r1, r2, r3], [r1, r_old, r3], [r2, r1]]
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        for ds in ((0, 0), (60, 3)):
            g, o = run_both(ctx, ss, agg=agg, ds_interval=ds[0], ds_agg=ds[1], exact=True)
            assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("seed,p_short", [(11, 0.5), (12, 1.0), (13, 0.15), (14, 0.85)])
def test_hourly_row_pairs(ctx, seed, p_short):
    """Spans of many hourly rows where a row whose cells end within 496 s of
    the hour merges into the RowSeq its predecessor started (Span.java:117,
    last - base < 4096), so merges alternate along runs of such rows; runs
    cross the 64-row batches of the wave walk. The last span also holds a
    row two hours on (no merge), and one span repeats a row (slow walk)."""
    T = T0
    rng = np.random.default_rng(seed)
    spans = []
    for n_rows in (150, 129, 65, 64, 3):
        rows = []
        for k in range(n_rows):
            base = T + 3600 * k
            hi = 490 if rng.random() < p_short else 3599
            offs = sorted(set(int(x) for x in rng.integers(0, hi + 1, 6)))
            rows.append(synth.compact_cells(base, [(base + o, 0x7, int(rng.integers(-1 << 40, 1 << 40)).to_bytes(
                8, "big", signed=True)) for o in offs]))
        spans.append(rows)
    b = T + 3600 * 151
    spans[-1] = spans[-1] + [synth.compact_cells(b, [(b + 5, 0x0, bytes([3]))])]
    spans.append(spans[1][:71] + [spans[1][70]] + spans[1][71:])
    ss = packing.pack_spans(spans)
    for agg in AGGS:
        for ds in ((0, 0), (600, 3)):
            g, o = run_both(ctx, ss, agg=agg, ds_interval=ds[0], ds_agg=ds[1], exact=True)
            assert_same(g, o, exact_double=True)


def test_short_overflow_merged_rowseq(ctx):
    """RowSeq.Iterator's short value_index overflows past 32767 value bytes."""
    T = T0
    r1 = synth.compact_cells(T, [(T + i, 0x7, int(i).to_bytes(8, "big")) for i in range(3600)])
    r2 = synth.compact_cells(T + 3600, [(T + 3600 + i, 0x7, int(i).to_bytes(8, "big")) for i in range(496)])
    ss = packing.pack_spans([[r1, r2]])
    g, o = run_both(ctx, ss)
    assert_same(g, o)
    assert g[0] == o.code


def test_device_generator_matches_host(ctx):
    import ctypes as C
    from opentsdb_amd import _lib
    L = _lib.lib()
    for kind in (_abi.SYN_INT64_COUNTER, _abi.SYN_FLOAT32, _abi.SYN_FLOAT64):
        host = synth.regular(7, 5000, kind, seed=11, step=5)
        p = _abi.SynthParams(seed=11, n_spans=7, n_points=5000, t0=T0, step=5, kind=kind)
        d = _abi.SgDesc()
        ctx.check(L.tsdbhip_synth_generate(ctx.handle, C.byref(p), C.byref(d)))
        R = d.n_rows
        arrs = [np.zeros(7 + 1, np.uint64), np.zeros(R, np.uint32), np.zeros(R, np.uint32),
                np.zeros(R, np.uint64), np.zeros(R, np.uint64), np.zeros(R, np.uint32),
                np.zeros(d.qual_nbytes, np.uint8), np.zeros(d.val_nbytes, np.uint8)]
        ctx.check(L.tsdbhip_desc_download(ctx.handle, C.byref(d), *[a.ctypes.data for a in arrs]))
        for a, b in zip(arrs, [host.span_row_start, host.row_base, host.row_ncells, host.row_qual_off,
                               host.row_val_off, host.row_val_len, host.qual_bytes, host.val_bytes]):
            np.testing.assert_array_equal(a, b)
        # run on the device-resident desc and compare with the oracle
        rc, ts, isi, bits, n_in, _ = core.run_spanset(ctx, host, 0, U32MAX, 0, False, 60, 3, device_desc=d)
        import oracle
        o = oracle.spangroup(host, 0, U32MAX, 0, False, 60, 3)
        assert_same((rc, ts, isi, bits, n_in, -1), o)
        L.tsdbhip_synth_free(ctx.handle, C.byref(d))


def test_spangroup_api_lazy_errors(ctx):
    T = T0
    sg = core.SpanGroup(None, 0, U32MAX, [core.Span(I([(T + 1, 1), (T + 2, 2)])),
                                          core.Span(F([(T + 1, 1.0), (T + 3, float("nan"))]))],
                        False, core.Aggregators.get("sum"), ctx=ctx)
    pts = []
    with pytest.raises(core.IllegalStateException):
        for dp in sg:
            pts.append(dp)
    import oracle
    o = oracle.spangroup(packing.pack_spans([s.rows for s in sg.spans]), 0, U32MAX, 0)
    assert len(pts) == len(o.ts)
