"""Output formatting: tsdbhip_format_points writes
what GraphHandler.respondAsciiQuery, Plot.dumpToFiles and CliQuery print per
DataPoint. Host code in libtsdbhip.so — runs on CPU.

Pinning: Double.toString values the JDK documents or that are well known
(JDK 19+ shortest-digit specification: Double.MIN_VALUE -> "4.9E-324",
1.0E23, 2.0E23, the 1e-3 / 1e7 notation switch), java.util.Formatter "%f"
(HALF_UP at six places of the decimal digits), and an independent Python
restatement (repr() digits + the same notation rules) on random doubles."""
import math
import struct

import numpy as np
import pytest

from opentsdb_amd import core


def dbits(v):
    return struct.unpack("<q", struct.pack("<d", v))[0]


def fmt_doubles(vals, mode=core.FMT_GNUPLOT):
    n = len(vals)
    out = core.format_points(mode, np.zeros(n, np.int64), np.zeros(n, np.uint8),
                             np.array([dbits(v) for v in vals], np.int64), metric="m")
    lines = out.splitlines()
    assert len(lines) == n
    return [l.split(" ")[-1] if mode == core.FMT_GNUPLOT else l.split(" ")[2] for l in lines]


JDK_KNOWN = [
    (4.9e-324, "4.9E-324"),            # Double.MIN_VALUE (two digits, not "5.0E-324")
    (1.7976931348623157e308, "1.7976931348623157E308"),  # Double.MAX_VALUE
    (1e23, "1.0E23"), (2e23, "2.0E23"),
    (100.0, "100.0"), (1.5, "1.5"), (-2.25, "-2.25"), (0.0, "0.0"), (-0.0, "-0.0"),
    (0.001, "0.001"), (0.0009999, "9.999E-4"), (1e-4, "1.0E-4"),
    (9999999.0, "9999999.0"), (1e7, "1.0E7"), (12345678.9, "1.23456789E7"),
    (0.1 + 0.2, "0.30000000000000004"), (1.0 / 3, "0.3333333333333333"),
    (123456.789, "123456.789"), (2.0 ** 60, "1.152921504606847E18"),
]


@pytest.mark.parametrize("v,s", JDK_KNOWN)
def test_double_tostring_known(v, s):
    assert fmt_doubles([v]) == [s]


def py_java_double(v):
    """Independent restatement: repr() gives the shortest round-trip digits."""
    v = float(v)
    if v == 0:
        return "-0.0" if math.copysign(1, v) < 0 else "0.0"
    sign = "-" if v < 0 else ""
    a = abs(v)
    m, e = ("%r" % a).replace("E", "e").partition("e")[::2] if "e" in repr(a) else (repr(a), "0")
    # normalise repr to digits/exponent
    mant = m.replace(".", "")
    dot = m.index(".") if "." in m else len(m)
    exp10 = int(e) + dot - 1
    digits = mant.lstrip("0")
    exp10 -= len(mant) - len(mant.lstrip("0"))
    digits = digits.rstrip("0") or "0"
    if len(digits) == 1:  # at least two significant digits, closest
        t = "%.1e" % a
        digits = t[0] + t[2]
        exp10 = int(t[4:])
        digits = digits.rstrip("0") or "0"
    if 1e-3 <= a < 1e7:
        if exp10 >= 0:
            ip = (digits + "0" * (exp10 + 1))[:exp10 + 1]
            fp = digits[exp10 + 1:] or "0"
            return sign + ip + "." + fp
        return sign + "0." + "0" * (-exp10 - 1) + digits
    return sign + digits[0] + "." + (digits[1:] or "0") + "E" + str(exp10)


def test_double_tostring_random():
    rng = np.random.default_rng(7)
    vals = list(rng.standard_normal(3000) * 10.0 ** rng.integers(-12, 15, 3000))
    vals += list(np.float32(rng.standard_normal(2000) + 100).astype(np.float64))  # widened float32 (C2/C4)
    vals += [float(x) for x in rng.integers(-10**9, 10**9, 500)]
    vals += list(struct.unpack("<%dd" % 500, rng.integers(0, 2**63 - 1, 500).astype(np.int64).tobytes()))
    vals = [v for v in vals if math.isfinite(v)]
    got = fmt_doubles(vals)
    for v, g in zip(vals, got):
        assert g == py_java_double(v), (v, g)
        assert float(g.replace("E", "e")) == v  # round trip


def test_pct_f_half_up():
    vals = [0.125, 1.0000005, 2.5e-7, 5e-7, -4.9e-7, 123.456789, 1e20, 0.0, -0.0, 0.9999995, 99.99999949]
    got = fmt_doubles(vals, core.FMT_CLI)
    assert got == ["0.125000", "1.000001", "0.000000", "0.000001", "-0.000000", "123.456789",
                   "100000000000000000000.000000", "0.000000", "-0.000000", "1.000000", "99.999999"]


def test_line_layouts():
    ts = np.array([1356998400, 1356998460], np.int64)
    isi = np.array([1, 0], np.uint8)
    bits = np.array([-42, dbits(2.5)], np.int64)
    a = core.format_points(core.FMT_ASCII, ts, isi, bits, metric="sys.cpu", tags=" host=a dc=b")
    assert a == "sys.cpu 1356998400 -42 host=a dc=b\nsys.cpu 1356998460 2.5 host=a dc=b\n"
    g = core.format_points(core.FMT_GNUPLOT, ts, isi, bits, utc_offset=-3600)
    assert g == "1356994800 -42\n1356994860 2.5\n"
    c = core.format_points(core.FMT_CLI, ts, isi, bits, metric="sys.cpu", tags="{host=a}")
    assert c == "sys.cpu 1356998400 -42 {host=a}\nsys.cpu 1356998460 2.500000 {host=a}\n"
    assert core.format_points(core.FMT_ASCII, ts[:0], isi[:0], bits[:0], metric="m") == ""


def test_nan_throws_like_the_reference():
    ts = np.array([1, 2], np.int64)
    isi = np.array([0, 0], np.uint8)
    bits = np.array([dbits(1.0), dbits(float("nan"))], np.int64)
    for mode in (core.FMT_ASCII, core.FMT_GNUPLOT):
        with pytest.raises(core.IllegalStateException):
            core.format_points(mode, ts, isi, bits, metric="m")
    assert core.format_points(core.FMT_CLI, ts, isi, bits, metric="m").splitlines()[1].split(" ")[2] == "NaN"


def test_many_points_parallel_chunks():
    n = 300_000  # several 64k-point chunks, formatted by parallel threads
    rng = np.random.default_rng(1)
    ts = np.arange(n, dtype=np.int64) + 1356998400
    isi = (rng.random(n) < 0.5).astype(np.uint8)
    vals = rng.standard_normal(n) * 1000
    bits = np.where(isi == 1, rng.integers(-10**6, 10**6, n), vals.view(np.int64))
    out = core.format_points(core.FMT_ASCII, ts, isi, bits, metric="m", tags=" h=x").splitlines()
    assert len(out) == n
    for i in (0, 1, 65535, 65536, 131071, n - 1):
        t, v = out[i].split(" ")[1:3]
        assert int(t) == ts[i]
        assert (int(v) == bits[i]) if isi[i] else (v == py_java_double(vals[i]))
