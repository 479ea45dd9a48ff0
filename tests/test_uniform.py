"""The uniform path (uniform_run in api.hip): every kept span one row on one
cadence with one class key (x0, n, step, flags), proposed at assembly from
the qualifiers of cells 0, 1 and n-1 (ug_probe). The union grid is then that
cadence (SpanGroup.java:510-608) and the call skips the grid kernels and the
second host round trip: the lockstep reduction without downsampling, the
aligned-group reduction with it (k_ds_reg). Every case is compared with the
oracle (integers bit-exact, doubles at 1e-9 relative); the proposal's
failures — a middle qualifier off the cadence that only the streaming kernel
sees — fall back to the proven path and must give the same results and
errors (timing.paths: PATH_UNIFORM, PATH_UNIFORM_FALLBACK, PATH_DIRECT_REDO)."""
import pytest

from helpers import I, T0, U32MAX, assert_same, corrupt_qual, run_both, with_option
from opentsdb_amd import _abi, core, packing, synth

pytestmark = pytest.mark.gpu
I64, F32, F64 = _abi.SYN_INT64_COUNTER, _abi.SYN_FLOAT32, _abi.SYN_FLOAT64


@pytest.fixture(autouse=True)
def always(request):
    """small groups: "always" takes the lockstep reduction whatever the size"""
    yield from with_option(request, "lockstep", "always", "on")


def paths(c):
    return c.timing().paths


@pytest.mark.parametrize("kind", [I64, F32, F64])
@pytest.mark.parametrize("agg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_uniform_lockstep(ctx, kind, agg, rate):
    ss = synth.regular(150, 1300, kind, seed=6, step=2)
    g, o = run_both(ctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    if agg != 4 or rate:
        assert paths(ctx) & _abi.PATH_UNIFORM and paths(ctx) & _abi.PATH_LOCKSTEP
    elif kind == I64:  # integer dev: the sequential chains of k_ug_dev (bit-exact)
        assert paths(ctx) & _abi.PATH_UNIFORM and not paths(ctx) & _abi.PATH_LOCKSTEP
        assert_same(g, o, exact_double=True)


@pytest.mark.parametrize("n_spans", [1, 95, 96, 97, 1000])
@pytest.mark.parametrize("width", [8, 4])
def test_uniform_integer_dev_chains(ctx, n_spans, width):
    """k_ug_dev: one sequential Welford chain a grid point over the spans in
    span order (Aggregators.java:196-237), phases of 96 spans; bit-exact
    against the oracle, counters near 2^40 (8-byte) or past 2^16 (4-byte)"""
    if width == 8:
        ss = synth.regular(n_spans, 700, I64, seed=13, step=1)
    else:
        # (values past 2^16 and inside int32: every cell 4 bytes wide)
        ss = packing.pack_spans([I([(T0 + 2 * i, 1_000_000 + 13 * i * (s + 1) - 70_000 * (s % 3)) for i in range(300)])
                                 for s in range(n_spans)])
    g, o = run_both(ctx, ss, agg=4)
    assert_same(g, o, exact_double=True)
    assert paths(ctx) & _abi.PATH_UNIFORM


def test_uniform_integer_dev_broken_reruns(ctx):
    """a middle qualifier off the cadence: k_ug_dev's producers see it, the
    call runs again on the proven path"""
    ss = corrupt_qual(synth.regular(300, 1300, I64, seed=3, step=2), 201, 700, lambda q: q + 16)
    g, o = run_both(ctx, ss, agg=4)
    assert_same(g, o, exact_double=True)
    assert paths(ctx) & _abi.PATH_DIRECT_REDO


@pytest.mark.parametrize("agg", [0, 1, 2, 3])
@pytest.mark.parametrize("dsa", [0, 1, 2, 3])
def test_uniform_aligned_group(ctx, agg, dsa):
    ss = synth.regular(200, 3600, I64, seed=12, step=1)
    g, o = run_both(ctx, ss, 0, U32MAX, agg, False, 60, dsa)
    assert_same(g, o)
    p = paths(ctx)
    assert p & _abi.PATH_UNIFORM and p & _abi.PATH_ALIGNED_GROUP and not p & _abi.PATH_UNIFORM_FALLBACK


@pytest.mark.parametrize("what", ["delta+1", "float-flag", "width-4"])
def test_uniform_aligned_group_broken_falls_back(ctx, what):
    """a middle qualifier the proposal never read: k_ds_reg finds the span off
    the cadence, the group does not stand, the general path runs the call"""
    fn = {"delta+1": lambda q: q + 16, "float-flag": lambda q: q | 0x8, "width-4": lambda q: (q & ~0x7) | 0x3}[what]
    # (step 2: the shifted delta stays increasing; a duplicate timestamp in a
    # row is input the reference never produces, E_UNSORTED here)
    ss = corrupt_qual(synth.regular(120, 1800, I64, seed=2, step=2), 77, 900, fn)
    for agg in (0, 2):
        g, o = run_both(ctx, ss, 0, U32MAX, agg, False, 60, 3)
        assert_same(g, o)
        assert paths(ctx) & _abi.PATH_UNIFORM_FALLBACK


def test_uniform_not_proposed(ctx):
    """spans that propose no key or different keys: the general path alone
    (a window cutting the spans, minimal-width cells, a second row, phases)"""
    ss = synth.regular(60, 1000, I64, seed=2, step=1)
    for start, end in ((T0 + 10, U32MAX), (0, T0 + 500)):
        g, o = run_both(ctx, ss, start=start, end=end, agg=0)
        assert_same(g, o)
        assert not paths(ctx) & _abi.PATH_UNIFORM
    minimal = packing.pack_spans([I([(T0 + i, 7 * i + s) for i in range(300)]) for s in range(40)])
    two_rows = packing.pack_spans([I([(T0 + 3000 + i, i) for i in range(1200)], minimal=False) for _ in range(40)])
    phases = packing.pack_spans([I([(T0 + (s % 3) + 3 * i, i) for i in range(400)], minimal=False) for s in range(40)])
    for ss in (minimal, two_rows, phases):
        for dsi in (0, 60):
            g, o = run_both(ctx, ss, agg=0, ds_interval=dsi, ds_agg=3 if dsi else 0)
            assert_same(g, o)
            # (spans of two rows: the downsampled kernels take them, k_lockstep not)
            assert bool(paths(ctx) & _abi.PATH_UNIFORM) == (ss is two_rows and dsi > 0)


@pytest.mark.parametrize("kind", [F32, F64, I64])
@pytest.mark.parametrize("agg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("dsa", [0, 1, 3])
@pytest.mark.parametrize("dsi", [60, 10])
def test_uniform_e(ctx, kind, agg, dsa, dsi):
    """downsampled groups outside the aligned group (floats, dev, more than 64
    buckets a span): k_ds_reg writes each span's E on the key's buckets and
    G from the key, k_reduce finds every span aligned on every tile"""
    ss = synth.regular(150, 1300, kind, seed=6, step=2)
    g, o = run_both(ctx, ss, 0, U32MAX, agg, False, dsi, dsa)
    assert_same(g, o)
    p = paths(ctx)
    assert p & _abi.PATH_UNIFORM and not p & (_abi.PATH_UNIFORM_FALLBACK | _abi.PATH_LOCKSTEP)
    fap = kind == I64 and agg <= 3 and (1300 + dsi // 2 - 1) // (dsi // 2) <= 64
    assert bool(p & _abi.PATH_ALIGNED_GROUP) == fap


@pytest.mark.parametrize("kind", [F64, I64])
@pytest.mark.parametrize("agg", [0, 3, 4])
def test_uniform_e_many_rows(ctx, kind, agg):
    """C2's shape: a day of hourly rows a span (k_ds_reg's 4 waves a span),
    1-minute buckets"""
    ss = synth.regular(40, 8640, kind, seed=7, step=10)
    g, o = run_both(ctx, ss, 0, U32MAX, agg, False, 60, 3)
    assert_same(g, o)
    assert paths(ctx) & _abi.PATH_UNIFORM


@pytest.mark.parametrize("row", [0, 5, 23])
def test_uniform_e_broken_falls_back(ctx, row):
    """a qualifier off the cadence in some row of one span: k_ds_reg leaves
    the span out, the call runs again on the general path"""
    ss = corrupt_qual(synth.regular(40, 8640, F64, seed=8, step=10), 17, 100, lambda q: q + 16, row=row)
    for agg in (0, 4):
        g, o = run_both(ctx, ss, 0, U32MAX, agg, False, 60, 3)
        assert_same(g, o)
        assert paths(ctx) & _abi.PATH_UNIFORM_FALLBACK


def test_uniform_e_window(ctx):
    """a window cutting the spans proposes nothing; one holding them whole does"""
    ss = synth.regular(40, 8640, F64, seed=9, step=10)
    for start, end, uni in ((0, U32MAX, True), (0, T0 + 86390, True), (0, T0 + 86389, False), (T0 + 5, U32MAX, False)):
        g, o = run_both(ctx, ss, start, end, 0, False, 60, 3)
        assert_same(g, o)
        assert bool(paths(ctx) & _abi.PATH_UNIFORM) == uni


@pytest.fixture(scope="module", params=[2, 4, 8])
def mctx(request):
    from opentsdb_amd._lib import Context
    c = Context(devices=[0] * request.param)
    yield c
    c.close()


def both(c, ss, **kw):
    import oracle
    a = dict(start=0, end=U32MAX, agg=0, rate=False, dsi=0, dsa=0)
    a.update(kw)
    g = core.run_spanset(c, ss, a["start"], a["end"], a["agg"], a["rate"], a["dsi"], a["dsa"])
    o = oracle.spangroup(ss, a["start"], a["end"], a["agg"], a["rate"], a["dsi"], a["dsa"])
    return g, o


@pytest.mark.timeout(120)
@pytest.mark.parametrize("agg", [0, 2, 3, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_uniform_sharded_lockstep(mctx, agg, rate):
    """the ranks agree on the key before the round trip (one collective), the
    partials travel in a second one"""
    ss = synth.regular(8 * mctx.ranks, 900, I64, seed=4, step=1)
    g, o = both(mctx, ss, agg=agg, rate=rate)
    assert_same(g, o)
    if agg != 4 or rate:
        assert paths(mctx) & _abi.PATH_UNIFORM
        assert mctx.timing().n_collectives == 2


@pytest.mark.timeout(120)
@pytest.mark.parametrize("agg", [0, 1, 2, 3])
def test_uniform_sharded_aligned_group(mctx, agg):
    """the key agreement, the validity and the 64-slot partials in one collective"""
    ss = synth.regular(8 * mctx.ranks, 3600, I64, seed=9, step=1)
    g, o = both(mctx, ss, agg=agg, dsi=60, dsa=3)
    assert_same(g, o)
    assert paths(mctx) & _abi.PATH_UNIFORM and paths(mctx) & _abi.PATH_ALIGNED_GROUP
    assert mctx.timing().n_collectives == 1


@pytest.mark.timeout(120)
def test_uniform_sharded_ranks_on_other_keys(mctx):
    """each rank uniform on its own key (phases differ by rank): the agreement
    refuses the uniform path everywhere (lockstep) / the aligned group does
    not stand anywhere (downsampled), and the general path gives the results"""
    n = 4 * mctx.ranks
    spans = [I([(T0 + (s >= n // 2) + 2 * i, s * 7 + i) for i in range(900)], minimal=False) for s in range(n)]
    ss = packing.pack_spans(spans)
    g, o = both(mctx, ss, agg=0)
    assert_same(g, o)
    assert not paths(mctx) & _abi.PATH_UNIFORM
    g, o = both(mctx, ss, agg=2, dsi=60, dsa=3)
    assert_same(g, o)
    assert paths(mctx) & _abi.PATH_UNIFORM_FALLBACK


@pytest.mark.timeout(120)
def test_uniform_sharded_broken_in_one_rank(mctx):
    """a middle qualifier off the cadence in the last rank: lockstep reruns on
    the proven path, the aligned group falls back, every rank alike"""
    ss = corrupt_qual(synth.regular(8 * mctx.ranks, 1800, I64, seed=4, step=2), 8 * mctx.ranks - 1, 1000,
                      lambda q: q + 16)
    g, o = both(mctx, ss, agg=0)
    assert_same(g, o)
    assert paths(mctx) & _abi.PATH_DIRECT_REDO
    g, o = both(mctx, ss, agg=0, dsi=60, dsa=3)
    assert_same(g, o)
    assert paths(mctx) & _abi.PATH_UNIFORM_FALLBACK


@pytest.mark.timeout(180)
@pytest.mark.parametrize("dsi", [0, 60])
def test_uniform_sharded_many_spans_rank_shifted(mctx, dsi):
    """more than KC_MAX (4096) spans a rank, so the kept list goes through
    the tiled kernels (k_kept_tiles / k_kept_scatter_tiles, whose last block
    alone folds the key words: ADVICE r5), and the last rank's spans one row
    (3600 s) later than everyone else's: the key agreement must see the
    disagreement — lockstep refuses the uniform path, the aligned group does
    not stand — and the general path gives the oracle's results"""
    n = 4200 * mctx.ranks
    ss = synth.regular(n, 120, I64, seed=21, step=1)
    last = n - n // mctx.ranks  # (contiguous shards: the last rank's first span)
    r0 = int(ss.span_row_start[last])
    ss.row_base[r0:] += 3600
    g, o = both(mctx, ss, agg=0, dsi=dsi, dsa=3 if dsi else 0)
    assert_same(g, o)
    if dsi:
        assert paths(mctx) & _abi.PATH_UNIFORM_FALLBACK and not paths(mctx) & _abi.PATH_ALIGNED_GROUP
    else:
        assert not paths(mctx) & _abi.PATH_UNIFORM


@pytest.mark.timeout(120)
def test_uniform_sharded_fallback_stages_once(mctx):
    """a downsampled query whose aligned group does not stand reruns on the
    general path without copying its host-resident inputs again:
    the rerun's call copies as many bytes as a call that never tried"""
    n = 4 * mctx.ranks
    spans = [I([(T0 + (s >= n // 2) + 2 * i, s * 7 + i) for i in range(900)], minimal=False) for s in range(n)]
    ss = packing.pack_spans(spans)
    g, o = both(mctx, ss, agg=2, dsi=60, dsa=3)
    assert_same(g, o)
    assert paths(mctx) & _abi.PATH_UNIFORM_FALLBACK
    fell_back = mctx.timing().h2d_bytes
    g, o = both(mctx, ss, agg=2, dsi=60, dsa=4)  # (dev downsampling: no aligned-group attempt)
    assert_same(g, o)
    assert not paths(mctx) & _abi.PATH_UNIFORM_FALLBACK
    assert fell_back == mctx.timing().h2d_bytes > 0


@pytest.mark.parametrize("agg", [0, 4])
@pytest.mark.parametrize("dsi", [2700, 10800])
def test_uniform_e_buckets_across_pieces(ctx, agg, dsi):
    """the E variant's pieces (k_ds_reg waves a span) must each start on a
    bucket head: 45-minute and 3-hour buckets over 16 hourly rows of 1-s
    cells do not divide 8 rows, so the host picks fewer pieces and the call
    takes the uniform path without a fallback"""
    ss = synth.regular(12, 16 * 3600, F64, seed=23, step=1)
    g, o = run_both(ctx, ss, 0, U32MAX, agg, False, dsi, 3)
    assert_same(g, o)
    assert paths(ctx) & _abi.PATH_UNIFORM and not paths(ctx) & _abi.PATH_UNIFORM_FALLBACK
