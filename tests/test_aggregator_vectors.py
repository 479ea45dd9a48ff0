"""The reference's own Aggregators.StdDev vectors (TestAggregators.java:68-120:
dev of 0..9999, {3,3,3}, {1,2}; tests/golden/known_answers.json) through the
HIP path, not only the oracle, two ways each:

* one span of the values (ts T0 + i) downsampled by `dev` into one bucket
  (Span.DownsamplingIterator, Span.java:377-422: an all-int bucket runs
  ds.runLong, a float bucket ds.runDouble);
* as many one-point spans at one timestamp, aggregated by `dev` across the
  series (SpanGroup.SGIterator, SpanGroup.java:647-667).

Longs go through runLong (the (long) truncation of the sequential Welford,
Aggregators.java:196-217), doubles (8-byte float cells) through runDouble
(:219-238). Checked against the test's expected value with its epsilon
(runLong: max(epsilon, 1.0), as checkSimilarStdDev does) and bit-exactly
against the oracle."""
import json
import os
import struct

import pytest

import oracle
from helpers import F, I, T0, U32MAX, assert_same, run_both
from opentsdb_amd import _abi, packing

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "known_answers.json")))
DEV = _abi.AGG_DEV


def value_of(g, i=0):
    rc, ts, isi, bits, _, _ = g
    assert rc == 0
    return int(bits[i]) if isi[i] else struct.unpack("<d", struct.pack("<q", int(bits[i])))[0]


def one_span(values, double):
    pts = [(T0 + i, float(v) if double else int(v)) for i, v in enumerate(values)]
    return packing.pack_spans([F(pts, double=True) if double else I(pts, minimal=False)])


def point_spans(values, double):
    return packing.pack_spans([F([(T0, float(v))], double=True) if double else I([(T0, int(v))], minimal=False)
                               for v in values])


@pytest.mark.gpu
@pytest.mark.parametrize("case", GOLD["aggregators"], ids=lambda c: c["name"])
@pytest.mark.parametrize("double", [False, True])
@pytest.mark.parametrize("shape", ["downsample", "across_spans"])
def test_stddev_vectors_on_the_gpu(ctx, case, double, shape):
    vals = case["values"]
    if shape == "downsample":  # one bucket holding every value
        g, o = run_both(ctx, one_span(vals, double), agg=_abi.AGG_SUM, ds_interval=len(vals) + 1, ds_agg=DEV)
    else:
        g, o = run_both(ctx, point_spans(vals, double), agg=DEV)
    assert len(g[1]) == 1
    assert_same(g, o, exact_double=True)
    v = value_of(g)
    if double:
        assert isinstance(v, float) and abs(v - case["dev"]) <= case["eps"]
    else:
        assert isinstance(v, int) and abs(v - case["dev"]) <= max(case["eps"], 1.0)
        if "dev_long" in case:
            assert v == case["dev_long"]
