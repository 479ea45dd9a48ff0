"""The benchmarked configurations checked at their full size (VERDICT r1:
bench.py's own workloads were never validated).

* C3* / C3 (1M series x 3600 points @1 s, the device generator's bytes):
  tsdbhip_spangroup_run on the HBM-resident SpanGroup against the oracle run
  shard by shard on the host cores and combined in shard order
  (oracle.regular_sharded: sum / max over an aligned grid, where the per-shard
  outputs combine exactly; ints bit-exact, rate doubles at 1e-9 relative).
  Rate dev (Aggregators.java:219-238) combines the shards' Welford states
  pairwise in shard order (1e-9 relative).
* C2 (10k float32 series x 8640 points @10 s, avg + 1m-avg downsample, the
  device generator's bytes) against the whole-group oracle on the host
  generator's identical bytes (Span.java:377-422, Aggregators.java:150-175):
  1e-9 relative, and bit-exact under TSDBHIP_EXACT_ORDER.
* C4 / C4-int (synth.jittered_packed, the bench's generator) at a size whose
  union grid holds > 1M points over the 40M-s range, whole-group oracle; and
  at the bench's own size (1000 series, a ~10.5M-point union) against the
  digests of the whole-group oracle in tests/golden/fullsize_digests.json
  (tests/golden/make_fullsize_digests.py: ~3 min of oracle per case).
The CPU tests pin the sharded oracle against the plain oracle on
synth.regular at small sizes."""
import ctypes as C
import hashlib
import json
import os

import numpy as np
import pytest

import oracle
from helpers import U32MAX, assert_same
from opentsdb_amd import _abi, core, synth

I64, F32 = _abi.SYN_INT64_COUNTER, _abi.SYN_FLOAT32


# ------------------------------------------------------------------- CPU ----
@pytest.mark.parametrize("kind,step,agg,rate,dsi,dsa", [
    (I64, 1, _abi.AGG_SUM, False, 60, _abi.AGG_AVG),
    (I64, 1, _abi.AGG_SUM, False, 0, 0),
    (I64, 1, _abi.AGG_SUM, True, 0, 0),
    (I64, 1, _abi.AGG_MAX, True, 0, 0),
    (F32, 10, _abi.AGG_SUM, False, 60, _abi.AGG_AVG),
    (I64, 10, _abi.AGG_MIN, False, 60, _abi.AGG_SUM),
    (I64, 1, _abi.AGG_DEV, True, 0, 0),
    (F32, 10, _abi.AGG_DEV, False, 60, _abi.AGG_AVG),
])
def test_sharded_oracle_matches_whole_group(kind, step, agg, rate, dsi, dsa):
    """oracle_regular_sharded (C generator + shard combine) == the oracle on
    synth.regular's bytes for the whole group (sum of doubles: 1e-12)."""
    n_spans, n_points = 37, 2 * 3600 // step + 5
    whole = oracle.spangroup(synth.regular(n_spans, n_points, kind, seed=3, step=step), 0, U32MAX, agg, rate,
                             dsi, dsa)
    sh = oracle.regular_sharded(n_spans, n_points, kind, 3, step, 0, U32MAX, agg, rate, dsi, dsa,
                                shard_spans=5, threads=4)
    g = (sh.code, sh.ts, sh.is_int, sh.bits, sh.n_input_points, -1)
    assert_same(g, whole, rtol=1e-12)


def test_sharded_oracle_rejects_unaligned():
    assert oracle.regular_sharded(4, 100, I64, 1, 1, 0, U32MAX, _abi.AGG_AVG).code == _abi.E_INVALID_ARG
    # the long dev (no rate, int series) truncates a sequential Welford: no merge
    assert oracle.regular_sharded(4, 100, I64, 1, 1, 0, U32MAX, _abi.AGG_DEV).code == _abi.E_INVALID_ARG


DIGESTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize_digests.json")


def sha(a, dt):
    return hashlib.sha256(np.ascontiguousarray(a.astype(dt)).tobytes()).hexdigest()


def test_fullsize_digests_fixture():
    """The committed oracle digests describe bench.py's C4 workloads."""
    d = json.load(open(DIGESTS))
    for name in ("c4_sum", "c4i_sum", "c4_avg"):
        e = d[name]
        assert e["code"] == 0 and e["n_series"] == 1000 and e["n_points"] == 11500 and e["seed"] == 4
        assert e["n_out"] > 10_000_000 and e["n_input"] > 11_000_000


# ------------------------------------------------------------------- GPU ----
@pytest.fixture(scope="module")
def c3_desc(ctx):
    """C3 / C3*: 1M series x 3600 points @1 s, 8-byte counters, in HBM."""
    d = _abi.SgDesc()
    p = _abi.SynthParams(seed=3, n_spans=1_000_000, n_points=3600, t0=synth.T0, step=1, kind=I64, span0=0)
    ctx.check(ctx._lib.tsdbhip_synth_generate(ctx.handle, C.byref(p), C.byref(d)))
    yield d
    ctx._lib.tsdbhip_synth_free(ctx.handle, C.byref(d))


def run_device(ctx, d, agg, rate=False, dsi=0, dsa=0, cap=3600, exact=False):
    d.start_time, d.end_time = 0, U32MAX
    d.agg, d.rate, d.ds_interval, d.ds_agg = agg, int(rate), dsi, dsa
    d.flags = _abi.DESC_DEVICE | (_abi.EXACT_ORDER if exact else 0)
    ts, isi, bits = np.zeros(cap, np.int64), np.zeros(cap, np.uint8), np.zeros(cap, np.int64)
    out = _abi.SgOut(capacity=cap, ts=_abi.ptr(ts, C.c_int64), is_int=_abi.ptr(isi, C.c_uint8),
                     bits=_abi.ptr(bits, C.c_int64))
    rc = ctx._lib.tsdbhip_spangroup_run(ctx.handle, C.byref(d), C.byref(out))
    n = int(out.n_out)
    return rc, ts[:n], isi[:n], bits[:n], int(out.n_input_points), int(out.err_index)


C3_CASES = [
    ("C3* sum + 1m-avg (the bench line)", _abi.AGG_SUM, False, 60, _abi.AGG_AVG),
    ("C3 sum", _abi.AGG_SUM, False, 0, 0),
    ("C3 rate sum", _abi.AGG_SUM, True, 0, 0),
    ("C3 rate max", _abi.AGG_MAX, True, 0, 0),
    ("C3 rate dev", _abi.AGG_DEV, True, 0, 0),
]
_C3_ORACLE = {}


def c3_oracle(agg, rate, dsi, dsa):
    """the 1M-series oracle of one C3 case (host threads, ~1 min), computed
    once for the unsharded and the 8-rank test"""
    key = (agg, rate, dsi, dsa)
    if key not in _C3_ORACLE:
        o = oracle.regular_sharded(1_000_000, 3600, I64, 3, 1, 0, U32MAX, agg, rate, dsi, dsa, shard_spans=2000)
        assert o.code == 0 and o.n_input_points == 3_600_000_000
        assert len(o.ts) == (60 if dsi else 3599 if rate else 3600)
        _C3_ORACLE[key] = o
    return _C3_ORACLE[key]


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,agg,rate,dsi,dsa", C3_CASES)
def test_c3_full_size(ctx, c3_desc, name, agg, rate, dsi, dsa):
    g = run_device(ctx, c3_desc, agg, rate, dsi, dsa)
    assert_same(g, c3_oracle(agg, rate, dsi, dsa), rtol=1e-9)


@pytest.fixture(scope="module")
def ctx8():
    """8 in-process ranks on the one GPU (LocalXchg): the sharded path of
    bench.py --gpus 8 with every per-rank kernel, chunking and exchange step
    at the benchmarked per-rank size (125k spans a rank)"""
    from opentsdb_amd._lib import Context
    c = Context(devices=[0] * 8)
    assert c.ranks == 8
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,agg,rate,dsi,dsa", C3_CASES)
def test_c3_full_size_8_ranks(ctx8, c3_desc, name, agg, rate, dsi, dsa):
    """the series-sharded path at the C3 size (1M spans
    split over 8 ranks) against the same oracle: the per-rank
    reduce chunking, the optimistic aligned-group finish (C3*: asserted
    taken, one collective), exact integer partials allreduced, rate doubles
    gathered and merged in rank order (SpanGroup.java:647-667,736-784) at
    1e-9 relative, integers bit-exact."""
    g = run_device(ctx8, c3_desc, agg, rate, dsi, dsa)
    tm = ctx8.timing()
    assert_same(g, c3_oracle(agg, rate, dsi, dsa), rtol=1e-9)
    if dsi:
        assert tm.paths & _abi.PATH_ALIGNED_GROUP
        assert tm.n_collectives == 1


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("gen,agg", [("c4", _abi.AGG_SUM), ("c4", _abi.AGG_AVG), ("c4i", _abi.AGG_SUM),
                                     ("c4i", _abi.AGG_DEV), ("c4i", _abi.AGG_MIN)])
def test_c4_million_point_union(ctx, gen, agg):
    """bench.py's C4 generator (jittered gaps U{1..6960} s, variable starts
    over a 40M-s range, mixed int/float32 or all-int) with 100 series of
    ~11.5k points: a union grid of > 1M points, general (bitmap + E) path."""
    ff, fc = (0.5, 0.01) if gen == "c4" else (0.0, 0.0)
    ss = synth.jittered_packed(100, 11500, seed=4, float_frac=ff, float_cell_frac=fc)
    # (registered result buffers: the reduce writes the results into them)
    g = core.run_spanset(ctx, ss, 0, U32MAX, agg, register_out=True)
    o = oracle.spangroup(ss, 0, U32MAX, agg, capacity=ss.n_cells() + 16)
    assert o.code == 0 and len(o.ts) > 1_000_000
    assert_same(g, o, abs_scale=abs_bound(100, 11500, 4, ff, fc, agg, o.ts))


def as_values(isi, bits):
    return np.where(isi.astype(bool), bits.astype(np.float64), bits.view(np.float64))


def abs_bound(n_series, n_points, seed, ff, fc, agg, ts):
    """Per output point, the oracle's aggregation over the |values| of the
    same series (synth.jittered_packed(absval=True)): an upper bound of the
    aggregated |terms| a mixed-sign double sum is rounded against (SURVEY.md
    §8(d): C4's tolerance is relative to sum|x|, not to a result that can
    cancel to ~0). From the CPU oracle, so no GPU result sets its own
    tolerance."""
    sa = synth.jittered_packed(n_series, n_points, seed=seed, float_frac=ff, float_cell_frac=fc, absval=True)
    o = oracle.spangroup(sa, 0, U32MAX, agg, capacity=sa.n_cells() + 16)
    assert o.code == 0 and np.array_equal(o.ts, ts)
    return as_values(o.is_int, o.bits)


def abs_bound_full(ctx, e, name):
    """abs_bound at the bench's own size (1000 series, where the oracle takes
    ~3 min): the GPU's EXACT_ORDER run of the |values| group, accepted only
    once it matches the oracle's digest of that run bit for bit
    (tests/golden/fullsize_digests.json, "<name>_abs")."""
    d = json.load(open(DIGESTS))[name + "_abs"]
    ff, fc = (0.5, 0.01) if e["gen"] == "jitter" else (0.0, 0.0)
    sa = synth.jittered_packed(e["n_series"], e["n_points"], seed=e["seed"], float_frac=ff, float_cell_frac=fc,
                               absval=True)
    rc, ts, isi, bits, _, _ = core.run_spanset(ctx, sa, 0, U32MAX, e["agg"], exact=True)
    assert rc == d["code"] and len(ts) == d["n_out"]
    assert sha(ts, "<i8") == d["ts"] and sha(isi, "u1") == d["is_int"] and sha(bits, "<i8") == d["bits"], \
        "the |values| run differs from the oracle's digest"
    return as_values(isi, bits)


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_c2_full_size(ctx):
    """configs[1] at its size: 10k float32 series x 1 day @10 s, avg with
    1m-avg downsampling (the device generator's bytes, bench.py --config c2),
    whole-group oracle on synth.regular's identical bytes."""
    d = _abi.SgDesc()
    p = _abi.SynthParams(seed=3, n_spans=10_000, n_points=8640, t0=synth.T0, step=10, kind=F32, span0=0)
    ctx.check(ctx._lib.tsdbhip_synth_generate(ctx.handle, C.byref(p), C.byref(d)))
    try:
        g = run_device(ctx, d, _abi.AGG_AVG, False, 60, _abi.AGG_AVG, cap=2000)
        gx = run_device(ctx, d, _abi.AGG_AVG, False, 60, _abi.AGG_AVG, cap=2000, exact=True)
    finally:
        ctx._lib.tsdbhip_synth_free(ctx.handle, C.byref(d))
    ss = synth.regular(10_000, 8640, F32, seed=3, step=10)
    o = oracle.spangroup(ss, 0, U32MAX, _abi.AGG_AVG, False, 60, _abi.AGG_AVG, capacity=2000)
    del ss
    assert o.code == 0 and o.n_input_points == 86_400_000 and len(o.ts) == 1440
    assert not o.is_int.any()
    assert_same(g, o, rtol=1e-9)
    assert_same(gx, o, exact_double=True)


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["c4_sum", "c4i_sum", "c4_avg"])
def test_c4_full_size(ctx, name):
    """bench.py's C4 / C4-int line at its own size (1000 jittered series,
    ~11.7M cells, a ~10.5M-point union grid; SpanGroup.java:702-784 lerps)
    against the whole-group oracle's digests: timestamps, isInteger and the
    long values bit-exactly; doubles bit-exactly under TSDBHIP_EXACT_ORDER and
    within 1e-9 of that run in the default (chunk-parallel) order."""
    e = json.load(open(DIGESTS))[name]
    ff, fc = (0.5, 0.01) if e["gen"] == "jitter" else (0.0, 0.0)
    ss = synth.jittered_packed(e["n_series"], e["n_points"], seed=e["seed"], float_frac=ff, float_cell_frac=fc)
    gx = core.run_spanset(ctx, ss, 0, U32MAX, e["agg"], exact=True)
    g = core.run_spanset(ctx, ss, 0, U32MAX, e["agg"], register_out=True)
    rc, ts, isi, bits, n_in, _ = gx
    assert rc == e["code"] and n_in == e["n_input"] and len(ts) == e["n_out"]
    assert sha(ts, "<i8") == e["ts"], "timestamps differ from the oracle"
    assert sha(isi, "u1") == e["is_int"], "isInteger differs from the oracle"
    assert sha(bits, "<i8") == e["bits"], "value bits (EXACT_ORDER) differ from the oracle"
    sc = abs_bound_full(ctx, e, name) if e["gen"] == "jitter" else None
    assert_same(g, oracle.Result(0, ts, isi, bits, n_in, -1), rtol=1e-9, abs_scale=sc)


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["c4_sum", "c4_avg"])
def test_c4_full_size_8_ranks_sliced(ctx, ctx8, name):
    """C4 at the bench's size over 8 ranks in the default order: the double
    partials travel as rank-owned slices of the ~10.5M-point grid (alltoall,
    rank-ordered merge, gathered results; SpanGroup.java:647-667). Timestamps
    and isInteger against the oracle's digests; values within 1e-9 of the
    oracle-verified sum of |terms|; the bytes each rank received against the
    slice exchange's size."""
    e = json.load(open(DIGESTS))[name]
    ss = synth.jittered_packed(e["n_series"], e["n_points"], seed=e["seed"], float_frac=0.5, float_cell_frac=0.01)
    g = core.run_spanset(ctx8, ss, 0, U32MAX, e["agg"])
    x_bytes = ctx8.timing().x_bytes
    rc, ts, isi, bits, n_in, _ = g
    assert rc == e["code"] and n_in == e["n_input"] and len(ts) == e["n_out"]
    assert sha(ts, "<i8") == e["ts"] and sha(isi, "u1") == e["is_int"]
    gx = core.run_spanset(ctx, ss, 0, U32MAX, e["agg"], exact=True)
    assert sha(gx[3], "<i8") == e["bits"]
    assert_same(g, oracle.Result(0, gx[1], gx[2], gx[3], gx[4], -1), rtol=1e-9, abs_scale=abs_bound_full(ctx, e, name))
    T = len(ts)
    # partials (cnt 4 + flag 1 + long 8 + double 8 B a point) once over the
    # slices, the 17-B results once, the grid bitmaps (1 bit a second of the
    # group's range) gathered; the allgather of every rank's partials would
    # be 7 x T x 21 B
    bitmap = 7 * ((int(ss.row_base.max()) + 3600 - int(ss.row_base.min())) // 32 + 2) * 4
    lo_x = 7 * ((T + 7) // 8) * (21 + 17)
    assert lo_x <= x_bytes <= lo_x + bitmap + 65536, (x_bytes, lo_x, bitmap)
    assert x_bytes < 7 * T * 21 / 3


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name", ["c4_sum", "c4i_sum"])
def test_c4_full_size_8_ranks(ctx8, name):
    """C4 / C4-int at the bench's size split over 8 in-process ranks: every
    rank's grid differs (bitmaps exchanged), the double partials are merged in
    rank order; under EXACT_ORDER the ranks form the span-ordered pipeline,
    bit-exact against the whole-group oracle's digests (SpanGroup.java:647-667)."""
    e = json.load(open(DIGESTS))[name]
    ff, fc = (0.5, 0.01) if e["gen"] == "jitter" else (0.0, 0.0)
    ss = synth.jittered_packed(e["n_series"], e["n_points"], seed=e["seed"], float_frac=ff, float_cell_frac=fc)
    rc, ts, isi, bits, n_in, _ = core.run_spanset(ctx8, ss, 0, U32MAX, e["agg"], exact=True)
    assert rc == e["code"] and n_in == e["n_input"] and len(ts) == e["n_out"]
    assert sha(ts, "<i8") == e["ts"], "timestamps differ from the oracle"
    assert sha(isi, "u1") == e["is_int"], "isInteger differs from the oracle"
    assert sha(bits, "<i8") == e["bits"], "value bits (EXACT_ORDER, 8 ranks) differ from the oracle"
