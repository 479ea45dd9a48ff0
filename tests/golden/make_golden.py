#!/usr/bin/env python3
"""Writes tests/golden/known_answers.json — the fixtures that pin the oracle.

Nothing here is computed by the oracle or the GPU path. The expected values
are the reference's own test vectors and hand-derived known answers:
  * TestAggregators.java:68-109 (dev on 0..9999, {3,3,3}, {1,2});
  * TestCompactionQueue.java:77-299 (the ten byte-exact compaction vectors,
    KEY-independent: compacted[0]'s qualifier/value bytes, and the put /
    delete calls each test verifies);
  * KA-1..KA-8 of SURVEY.md §8(c), traced by hand through
    SpanGroup.java:435-784 / Span.java:377-511 (KA-3/KA-6 re-derived here
    with absolute timestamps: the rate quirk Q5 divides by x0 itself).
The Java reference cannot run in this image (no JVM, jars not vendored), so
these literal expectations are the parity anchor.
"""
import json
import os
import struct

T = 1356998400


def L(v):
    return struct.pack(">q", v).hex()


def I4(v):
    return struct.pack(">i", v).hex()


def fbits(f):
    return struct.unpack(">I", struct.pack(">f", f))[0]


def spangroups():
    # series: list of [ts, "l"|"f"|"d", value]; expected: list of [ts, "l"|"d", value]
    return [
        {"name": "KA-1 int lerp sum", "agg": "sum",
         "spans": [[[T + 100, "l", 10], [T + 110, "l", 20]], [[T + 105, "l", 100], [T + 115, "l", 200]]],
         "expected": [[T + 100, "l", 10], [T + 105, "l", 115], [T + 110, "l", 170], [T + 115, "l", 200]]},
        {"name": "KA-2 truncation toward zero + lagged expiry", "agg": "sum",
         "spans": [[[T + 100, "l", 0], [T + 103, "l", -10]], [[T + 101, "l", 5]]],
         "expected": [[T + 100, "l", 0], [T + 101, "l", 2], [T + 103, "l", -10]]},
        {"name": "KA-8 bracket beyond end", "agg": "sum", "end": T + 160,
         "spans": [[[T + 100, "l", 0], [T + 200, "l", 100]], [[T + 150, "l", 7]]],
         "expected": [[T + 100, "l", 0], [T + 150, "l", 57]]},
        {"name": "KA-3 rate + Q5 (absolute ts)", "agg": "sum", "rate": True,
         "spans": [[[T + 100, "l", 10], [T + 110, "l", 30], [T + 120, "l", 60]],
                   [[T + 105, "l", 1000], [T + 115, "l", 1100]]],
         "expected": [[T + 110, "d", 2.0 + 1000.0 / float(T + 105)], [T + 115, "d", 12.0],
                      [T + 120, "d", 3.0]]},
        {"name": "KA-4 aligned 60s avg downsample", "agg": "sum", "ds": [60, "avg"],
         "spans": [[[T + 100 + i, "l", i] for i in range(120)]],
         "expected": [[T + 129, "l", 29], [T + 189, "l", 89]]},
        {"name": "KA-5 greedy buckets", "agg": "sum", "ds": [60, "sum"],
         "spans": [[[T + 100, "l", 1], [T + 130, "l", 2], [T + 161, "l", 3], [T + 170, "l", 4], [T + 230, "l", 5]]],
         "expected": [[T + 115, "l", 3], [T + 165, "l", 7], [T + 230, "l", 5]]},
        {"name": "KA-6 Q3 later float span forces double path", "agg": "sum",
         "spans": [[[T + 100, "l", 1], [T + 110, "l", 2]], [[T + 200, "f", 1.5], [T + 210, "f", 2.5]]],
         "expected": [[T + 100, "d", 1.0], [T + 110, "d", 2.0], [T + 200, "d", 1.5], [T + 210, "d", 2.5]]},
    ]


def compaction():
    # "put": whether tsdb.put(KEY, qual, val) is verified once (times(1)) or
    # never; "delete": the KVs (indices into "kvs") of the verified
    # tsdb.delete(KEY, new byte[][] {...}) call, [] for never() — both read
    # off the test's verify() lines (TestCompactionQueue.java:84-86, 98-100,
    # 116-119, 138-141, 162-165, 201-203, 227-230, 262-265, 294-298); an
    # expected exception (:168) means neither.
    q1, q2, q3 = "0007", "0027", "0017"
    return [
        {"name": "emptyRow", "kvs": [], "status": "none", "put": False, "delete": []},
        {"name": "oneCellRow", "kvs": [["0003", L(42)]], "status": "single", "qual": "0003", "val": L(42),
         "put": False, "delete": []},
        {"name": "twoCellRow", "kvs": [["0007", L(4)], ["0017", L(5)]], "status": "trivial",
         "qual": "00070017", "val": L(4) + L(5) + "00", "put": True, "delete": [0, 1]},
        {"name": "fixQualifierFlags", "kvs": [["0003", L(4)], ["0017", L(5)]], "status": "trivial",
         "qual": "00070017", "val": L(4) + L(5) + "00", "put": True, "delete": [0, 1]},
        {"name": "fixFloatingPoint", "kvs": [["0007", L(4)], ["001b", L(fbits(4.2))]], "status": "trivial",
         "qual": "0007001b", "val": L(4) + I4(fbits(4.2)) + "00", "put": True, "delete": [0, 1]},
        {"name": "overlappingDataPoints", "kvs": [["0007", L(4)], ["0003", I4(4)]], "status": "error",
         "put": False, "delete": []},
        {"name": "failedCompactNoop", "kvs": [[q1, L(4)], [q3, L(5)], [q1 + q3, L(4) + L(5) + "00"]],
         "status": "complex", "qual": q1 + q3, "val": L(4) + L(5) + "00", "put": False, "delete": [0, 1]},
        {"name": "secondCompact", "kvs": [[q1 + q2, L(4) + L(5) + "00"], [q3, L(6)]], "status": "complex",
         "qual": q1 + q3 + q2, "val": L(4) + L(6) + L(5) + "00", "put": True, "delete": [0, 1]},
        {"name": "doubleFailedCompactNoop",
         "kvs": [[q1, L(4)], [q1 + q3 + q2, L(4) + L(6) + L(5) + "00"], [q1 + q2, L(4) + L(5) + "00"],
                 [q3, L(6)], [q2, L(5)]],
         "status": "complex", "qual": q1 + q3 + q2, "val": L(4) + L(6) + L(5) + "00", "put": False,
         "delete": [0, 2, 3, 4]},
        {"name": "weirdOverlappingCompactedCells",
         "kvs": [[q1, L(4)], [q1 + q2, L(4) + L(5) + "00"], [q1 + q3, L(4) + L(6) + "00"], [q3, L(6)],
                 [q2, L(5)]],
         "status": "complex", "qual": q1 + q3 + q2, "val": L(4) + L(6) + L(5) + "00", "put": True,
         "delete": [0, 1, 2, 3, 4]},
    ]


def aggregators():
    return [
        {"name": "testStdDevKnownValues", "values": list(range(10000)), "dev": 2886.7513315143719,
         "eps": 0.01},
        {"name": "testStdDevNoDeviation", "values": [3, 3, 3], "dev": 0.0, "eps": 0.0, "dev_long": 0},
        {"name": "testStdDevFewDataInputs", "values": [1, 2], "dev": 0.5, "eps": 0.0, "dev_long": 0},
    ]


def main():
    out = {"source": __doc__.strip().splitlines()[0], "T0": T, "spangroups": spangroups(),
           "compaction": compaction(), "aggregators": aggregators()}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "known_answers.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
