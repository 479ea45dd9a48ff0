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

Usage: python tests/golden/make_fullsize_digests.py   (from the repo root)
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

# (name, generator, aggregator): bench.py's C4 lines
CASES = [("c4_sum", "jitter", 0), ("c4i_sum", "jitter_int", 0), ("c4_avg", "jitter", 3)]
N_SERIES, N_POINTS, SEED = 1000, 11500, 4


def spanset(gen):
    from opentsdb_amd import synth
    ff, fc = (0.5, 0.01) if gen == "jitter" else (0.0, 0.0)
    return synth.jittered_packed(N_SERIES, N_POINTS, seed=SEED, float_frac=ff, float_cell_frac=fc)


def digest(ts, isi, bits):
    import numpy as np
    h = lambda a: hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()  # noqa: E731
    return {"n_out": int(len(ts)), "ts": h(ts.astype("<i8")), "is_int": h(isi.astype("u1")),
            "bits": h(bits.astype("<i8")), "n_int": int(isi.astype(bool).sum())}


def one(case):
    import oracle
    from opentsdb_amd import _abi
    name, gen, agg = case
    ss = spanset(gen)
    t = time.time()
    o = oracle.spangroup(ss, 0, (1 << 32) - 1, agg, capacity=ss.n_cells() + 16)
    d = digest(o.ts, o.is_int, o.bits)
    d.update(code=int(o.code), n_input=int(o.n_input_points), gen=gen, agg=agg, n_series=N_SERIES,
             n_points=N_POINTS, seed=SEED, oracle_s=round(time.time() - t, 1))
    return name, d


def main():
    out = {"about": "sha256 of the oracle's (ts int64 LE, is_int u8, bits int64 LE) arrays on bench.py's C4 "
                    "workloads at full size; made by tests/golden/make_fullsize_digests.py"}
    with ProcessPoolExecutor(max_workers=len(CASES)) as ex:
        for name, d in ex.map(one, CASES):
            out[name] = d
            print(name, d, flush=True)
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "fullsize_digests.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
