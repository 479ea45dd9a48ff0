"""CPU: pin the oracle (oracle/oracle.cc) against the reference's own test
vectors and the hand-derived known answers in tests/golden, then
cross-check it against an independent closed-form restatement on random
small SpanGroups."""
import json
import math
import os
import struct

import numpy as np
import pytest

import oracle
import closed_form
from helpers import I, F, M, T0, U32MAX
from opentsdb_amd import _abi, compaction, packing, synth

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))
AGG = {"sum": 0, "min": 1, "max": 2, "avg": 3, "dev": 4}
STATUS = {"none": _abi.ROW_NONE, "single": _abi.ROW_SINGLE, "trivial": _abi.ROW_TRIVIAL,
          "complex": _abi.ROW_COMPLEX, "error": _abi.ROW_ERROR, "oob": _abi.ROW_OOB}


def spans_from_golden(case):
    out = []
    for s in case["spans"]:
        pts = []
        for ts, kind, v in s:
            if kind == "l":
                pts.append((ts,) + synth.encode_long(int(v)))
            elif kind == "f":
                pts.append((ts,) + synth.encode_float(float(v)))
            else:
                pts.append((ts,) + synth.encode_double(float(v)))
        out.append(synth.series_rows(pts))
    return packing.pack_spans(out)


@pytest.mark.parametrize("case", GOLD["spangroups"], ids=lambda c: c["name"])
def test_oracle_known_answers(case):
    ss = spans_from_golden(case)
    ds = case.get("ds", [0, "sum"])
    r = oracle.spangroup(ss, case.get("start", 0), case.get("end", U32MAX), AGG[case["agg"]],
                         case.get("rate", False), ds[0], AGG[ds[1]])
    assert r.code == 0
    exp = case["expected"]
    assert [int(t) for t in r.ts] == [e[0] for e in exp]
    for i, (t, kind, v) in enumerate(exp):
        assert bool(r.is_int[i]) == (kind == "l"), (case["name"], i)
        if kind == "l":
            assert int(r.bits[i]) == v
        else:
            assert struct.unpack("<d", struct.pack("<q", int(r.bits[i])))[0] == v


@pytest.mark.parametrize("case", GOLD["aggregators"], ids=lambda c: c["name"])
def test_oracle_test_aggregators(case):
    v = oracle.agg_double(_abi.AGG_DEV, case["values"])
    assert abs(v - case["dev"]) <= case["eps"]
    if "dev_long" in case:
        assert oracle.agg_long(_abi.AGG_DEV, case["values"]) == case["dev_long"]


def test_oracle_stddev_random_values_seeded():
    """TestAggregators.testStdDevRandomValues with a fixed seed: Welford vs
    a naive two-pass population deviation at 1e-4 relative."""
    rng = np.random.default_rng(1234)
    vals = [int(x) for x in rng.integers(-(1 << 62), 1 << 62, 1000)]
    mean = sum(float(x) for x in vals) / len(vals)
    naive = math.sqrt(sum((float(x) - mean) ** 2 for x in vals) / len(vals))
    assert abs(oracle.agg_double(_abi.AGG_DEV, vals) - naive) <= 1e-4 * naive


@pytest.mark.parametrize("case", GOLD["compaction"], ids=lambda c: c["name"])
def test_oracle_compaction_vectors(case):
    rows = [[(bytes.fromhex(q), bytes.fromhex(v)) for q, v in case["kvs"]]]
    res = oracle.compact_rows(compaction.pack_rows(rows))
    st, q, v = res.row(0)
    assert st == STATUS[case["status"]]
    if "qual" in case:
        assert q.hex() == case["qual"] and v.hex() == case["val"]
    # the put / delete calls the test verifies (write-back of an old row)
    put, dele = res.decision(0, [len(k) for k, _ in rows[0]])
    assert put == case["put"] and dele == case["delete"]


def _random_group(rng, n_spans, mixed, minimal):
    spans = []
    for _ in range(n_spans):
        n = int(rng.integers(1, 40))
        start = T0 + int(rng.integers(0, 4000))
        ts = start + np.cumsum(rng.integers(1, 300, n)) - 1
        pts = []
        is_float_series = mixed and rng.random() < 0.3
        for t in ts:
            if is_float_series:
                pts.append((int(t),) + synth.encode_float(float(rng.integers(-50, 50)) / 4))
            elif mixed and rng.random() < 0.05:
                pts.append((int(t),) + synth.encode_double(float(rng.integers(-1000, 1000)) / 8))
            else:
                pts.append((int(t),) + synth.encode_long(int(rng.integers(-10**9, 10**9)), minimal))
        spans.append(synth.series_rows(pts))
    return spans


@pytest.mark.parametrize("seed", range(24))
def test_oracle_matches_closed_form(seed):
    rng = np.random.default_rng(seed)
    spans = _random_group(rng, int(rng.integers(1, 7)), mixed=seed % 2 == 0, minimal=seed % 3 != 0)
    ss = packing.pack_spans(spans)
    for agg in range(5):
        for rate in (False, True):
            for interval, ds_agg in ((0, 0), (97, agg), (600, (agg + 2) % 5)):
                if rate and interval and seed % 4:
                    continue
                end = U32MAX if seed % 5 else T0 + 2500
                r = oracle.spangroup(ss, 0, end, agg, rate, interval, ds_agg)
                try:
                    exp = closed_form.spangroup(spans, 0, end, agg, rate, interval, ds_agg)
                    err = None
                except ArithmeticError as e:
                    exp, err = None, e.args[0]
                if err is not None:
                    assert r.code == _abi.E_NAN_INF and r.err_index == err
                    continue
                assert r.code == 0
                assert [int(x) for x in r.ts] == [e[0] for e in exp]
                for i, (t, isint, v) in enumerate(exp):
                    assert bool(r.is_int[i]) == isint
                    if isint:
                        assert int(r.bits[i]) == v
                    else:
                        got = struct.unpack("<d", struct.pack("<q", int(r.bits[i])))[0]
                        assert got == v or (got != got and v != v)


def test_synth_regular_layout():
    ss = synth.regular(3, 5000, _abi.SYN_FLOAT32, seed=2, step=10)
    assert ss.n_spans == 3 and ss.n_rows == 3 * 14
    rows = ss.span_rows(1)
    cells = closed_form.decode_cells(rows)
    assert len(cells) == 5000 and all(c[1] for c in cells)
    assert cells[0][0] == T0 and cells[1][0] - cells[0][0] == 10
    vals = np.array([c[2] for c in cells])
    assert 99.0 < vals.mean() < 101.0 and 0.8 < vals.std() < 1.2
    ci = synth.regular(2, 3600, _abi.SYN_INT64_COUNTER, seed=2, step=1)
    c = closed_form.decode_cells(ci.span_rows(0))
    d = np.diff([x[2] for x in c])
    assert (d > 0).all() and (d < 1000).all()
