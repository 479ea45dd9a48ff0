#!/usr/bin/env python3
"""Writes tests/golden/fullsize_digests.json: sha256 digests of the oracle's
output on the benchmarked C4 / C4-int workloads at their full size (1000
jittered series, ~11.7M cells, a ~10.5M-point union grid).

The oracle (oracle/oracle.cc, a line-by-line restatement of
SpanGroup.SGIterator, SpanGroup.java:370-796) needs ~3 minutes per case on
one core for these groups: too long for the GPU suite, so the digests are
computed here once and `tests/test_fullscale.py::test_c4_full_size` compares
the GPU output against them (timestamps, isInteger flags and value bits;
doubles bit-exactly under TSDBHIP_EXACT_ORDER, whose span-ordered sums are
the reference's order). The inputs are bench.py's own generator
(synth.jittered_packed, seed 4), deterministic across machines.

The "_abs" cases run the same groups on |value| (synth.jittered_packed
absval=True): their aggregate is the sum of |terms| the default-order
(chunk-parallel) double sums are checked against, so the
GPU's run of them is first matched bit-exactly (EXACT_ORDER) to these
digests and only then used as the tolerance scale.

Usage: python tests/golden/make_fullsize_digests.py [--force]   (from the repo root;
existing entries are kept unless --force)
"""
import hashlib
import json
import os
import sys
import time
from concurrent.futures import ProcessPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

# (name, generator, aggregator, |values|): bench.py's C4 lines, and the |terms| scales of
# the double-path ones
CASES = [("c4_sum", "jitter", 0, False), ("c4i_sum", "jitter_int", 0, False), ("c4_avg", "jitter", 3, False),
         ("c4_sum_abs", "jitter", 0, True), ("c4_avg_abs", "jitter", 3, True)]
N_SERIES, N_POINTS, SEED = 1000, 11500, 4


def spanset(gen, absval=False):
    from opentsdb_amd import synth
    ff, fc = (0.5, 0.01) if gen == "jitter" else (0.0, 0.0)
    return synth.jittered_packed(N_SERIES, N_POINTS, seed=SEED, float_frac=ff, float_cell_frac=fc, absval=absval)


def digest(ts, isi, bits):
    import numpy as np
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    return {"n_out": int(len(ts)), "ts": h(ts.astype("<i8")), "is_int": h(isi.astype("u1")),
            "bits": h(bits.astype("<i8")), "n_int": int(isi.astype(bool).sum())}


def one(case):
    import oracle
    from opentsdb_amd import _abi
    name, gen, agg, absval = case
    ss = spanset(gen, absval)
    t = time.time()
    o = oracle.spangroup(ss, 0, (1 << 32) - 1, agg, capacity=ss.n_cells() + 16)
    d = digest(o.ts, o.is_int, o.bits)
    d.update(code=int(o.code), n_input=int(o.n_input_points), gen=gen, agg=agg, n_series=N_SERIES,
             n_points=N_POINTS, seed=SEED, oracle_s=round(time.time() - t, 1), absval=absval)
    return name, d


def main():
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fullsize_digests.json")
    out = {}
    if os.path.exists(path) and "--force" not in sys.argv:
        out = json.load(open(path))
    out["about"] = ("sha256 of the oracle's (ts int64 LE, is_int u8, bits int64 LE) arrays on bench.py's C4 "
                    "workloads at full size (_abs: on |values|); made by tests/golden/make_fullsize_digests.py")
    todo = [c for c in CASES if c[0] not in out]
    with ProcessPoolExecutor(max_workers=max(1, len(todo))) as ex:
        for name, d in ex.map(one, todo):
            out[name] = d
            print(name, d, flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
