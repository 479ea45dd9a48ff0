"""The benchmarked configurations checked at their full size (VERDICT r1:
bench.py's own workloads were never validated).

* C3* / C3 (1M series x 3600 points @1 s, the device generator's bytes):
  tsdbhip_spangroup_run on the HBM-resident SpanGroup against the oracle run
  shard by shard on the host cores and combined in shard order
  (oracle.regular_sharded: sum / max over an aligned grid, where the per-shard
  outputs combine exactly; ints bit-exact, rate doubles at 1e-9 relative).
* C4 / C4-int (synth.jittered_packed, the bench's generator) at a size whose
  union grid holds > 1M points over the 40M-s range, whole-group oracle.
The CPU tests pin the sharded oracle against the plain oracle on
synth.regular at small sizes."""
import ctypes as C

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


# ------------------------------------------------------------------- GPU ----
@pytest.fixture(scope="module")
def c3_desc(ctx):
    """C3 / C3*: 1M series x 3600 points @1 s, 8-byte counters, in HBM."""
    d = _abi.SgDesc()
    p = _abi.SynthParams(seed=3, n_spans=1_000_000, n_points=3600, t0=synth.T0, step=1, kind=I64, span0=0)
    ctx.check(ctx._lib.tsdbhip_synth_generate(ctx.handle, C.byref(p), C.byref(d)))
    yield d
    ctx._lib.tsdbhip_synth_free(ctx.handle, C.byref(d))


def run_device(ctx, d, agg, rate=False, dsi=0, dsa=0, cap=3600):
    d.start_time, d.end_time = 0, U32MAX
    d.agg, d.rate, d.ds_interval, d.ds_agg = agg, int(rate), dsi, dsa
    ts, isi, bits = np.zeros(cap, np.int64), np.zeros(cap, np.uint8), np.zeros(cap, np.int64)
    out = _abi.SgOut(capacity=cap, ts=_abi.ptr(ts, C.c_int64), is_int=_abi.ptr(isi, C.c_uint8),
                     bits=_abi.ptr(bits, C.c_int64))
    rc = ctx._lib.tsdbhip_spangroup_run(ctx.handle, C.byref(d), C.byref(out))
    n = int(out.n_out)
    return rc, ts[:n], isi[:n], bits[:n], int(out.n_input_points), int(out.err_index)


@pytest.mark.gpu
@pytest.mark.timeout(600)
@pytest.mark.parametrize("name,agg,rate,dsi,dsa", [
    ("C3* sum + 1m-avg (the bench line)", _abi.AGG_SUM, False, 60, _abi.AGG_AVG),
    ("C3 sum", _abi.AGG_SUM, False, 0, 0),
    ("C3 rate sum", _abi.AGG_SUM, True, 0, 0),
    ("C3 rate max", _abi.AGG_MAX, True, 0, 0),
])
def test_c3_full_size(ctx, c3_desc, name, agg, rate, dsi, dsa):
    g = run_device(ctx, c3_desc, agg, rate, dsi, dsa)
    o = oracle.regular_sharded(1_000_000, 3600, I64, 3, 1, 0, U32MAX, agg, rate, dsi, dsa, shard_spans=2000)
    assert o.code == 0 and o.n_input_points == 3_600_000_000
    assert len(o.ts) == (60 if dsi else 3599 if rate else 3600)
    assert_same(g, o, rtol=1e-9)


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
    g = core.run_spanset(ctx, ss, 0, U32MAX, agg)
    o = oracle.spangroup(ss, 0, U32MAX, agg, capacity=ss.n_cells() + 16)
    assert o.code == 0 and len(o.ts) > 1_000_000
    assert_same(g, o)
