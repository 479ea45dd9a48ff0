"""Pure-Python closed form of the SpanGroup semantics (SURVEY.md §8a,
"closed-form restatement") — a second, independent restatement used only to
cross-check the iterator-faithful oracle on small random inputs. The GPU
kernels implement this closed form; the oracle implements the Java
iterators; agreement of the two on random inputs is what licenses the GPU
design. Small inputs only (pure-Python loops).
"""
import math
import struct

M64 = (1 << 64) - 1


def wrap(x):
    x &= M64
    return x - (1 << 64) if x >> 63 else x


def jdiv(a, b):  # Java long division (truncating)
    q = abs(a) // abs(b)
    return wrap(q if (a >= 0) == (b > 0) else -q)


def d2l(d):
    if d != d:
        return 0
    if d >= 9.223372036854775807e18:
        return (1 << 63) - 1
    if d <= -9.223372036854775808e18:
        return -(1 << 63)
    return int(d)


def agg_long(agg, vals):
    if agg == 0:
        r = vals[0]
        for v in vals[1:]:
            r = wrap(r + v)
        return r
    if agg == 1:
        m = vals[0]
        for v in vals[1:]:
            if v < m:
                m = v
        return m
    if agg == 2:
        m = vals[0]
        for v in vals[1:]:
            if v > m:
                m = v
        return m
    if agg == 3:
        r = vals[0]
        for v in vals[1:]:
            r = wrap(r + v)
        return jdiv(r, len(vals))
    return d2l(dev([float(v) for v in vals]))


def dev(xs):
    if len(xs) == 1:
        return 0.0
    mean, var, n = xs[0], 0.0, 2
    for x in xs[1:]:
        nm = mean + (x - mean) / n
        var += (x - mean) * (x - nm)
        mean = nm
        n += 1
    return math.sqrt(var / (n - 1))


def agg_double(agg, vals):
    if agg == 0:
        r = vals[0]
        for v in vals[1:]:
            r += v
        return r
    if agg == 1:
        m = vals[0]
        for v in vals[1:]:
            if v < m:
                m = v
        return m
    if agg == 2:
        m = vals[0]
        for v in vals[1:]:
            if v > m:
                m = v
        return m
    if agg == 3:
        r = vals[0]
        for v in vals[1:]:
            r += v
        return r / len(vals)
    return dev(vals)


def decode_cells(kvs):
    """Sorted, well-formed compacted rows of one span -> [(ts, is_float, value)]"""
    out = []
    for kv in kvs:
        off = 0
        for i in range(0, len(kv.qualifier), 2):
            q = (kv.qualifier[i] << 8) | kv.qualifier[i + 1]
            ln = (q & 7) + 1
            b = kv.value[off:off + ln]
            off += ln
            if q & 8:
                v = struct.unpack(">f", b)[0] if ln == 4 else struct.unpack(">d", b)[0]
                out.append((kv.base_time + (q >> 4), True, v))
            else:
                out.append((kv.base_time + (q >> 4), False, int.from_bytes(b, "big", signed=True)))
    return out


def emitted(cells, start, interval, ds_agg):
    """E_s: points >= start, greedily downsampled if interval > 0."""
    pts = [c for c in cells if c[0] >= start]
    if not interval:
        return pts
    out, i = [], 0
    while i < len(pts):
        end = pts[i][0] + interval
        j = i
        while j < len(pts) and pts[j][0] < end:
            j += 1
        b = pts[i:j]
        ts = sum(p[0] for p in b) // len(b)
        if all(not p[1] for p in b):
            out.append((ts, False, agg_long(ds_agg, [p[2] for p in b])))
        else:
            out.append((ts, True, agg_double(ds_agg, [float(p[2]) for p in b])))
        i = j
    return out


def spangroup(spans, start, end, agg, rate=False, interval=0, ds_agg=0):
    """spans: list of lists of KeyValue (well-formed, sorted, no Q1 seek).
    Returns list of (ts, is_int, value) or raises ArithmeticError for NaN/Inf."""
    E = []
    for kvs in spans:
        cells = decode_cells(kvs)
        if not cells or not (cells[0][0] <= end and cells[-1][0] >= start):
            continue
        E.append(emitted(cells, start, interval, ds_agg))
    if rate:
        G = sorted({p[0] for e in E if len(e) >= 2 for p in e[1:] if p[0] <= end})
    else:
        G = sorted({p[0] for e in E for p in e if p[0] <= end})
    out = []
    for t in G:
        if rate:
            vals = []
            for e in E:
                if len(e) < 2 or t > e[-1][0]:
                    continue
                idx = max([j for j in range(1, len(e)) if e[j][0] <= t], default=0)
                x0, _, y0 = e[idx]
                xp, yp = (0, 0.0) if idx == 0 else (e[idx - 1][0], float(e[idx - 1][2]))
                vals.append((float(y0) - yp) / float(x0 - xp))
            r = agg_double(agg, vals)
            if r != r or math.isinf(r):
                raise ArithmeticError(len(out))
            out.append((t, False, r))
            continue
        isf = False
        act = []
        for e in E:
            cur = max([j for j in range(len(e)) if e[j][0] <= t], default=-1)
            nxt = cur + 1
            active = cur >= 0 and t <= e[-1][0]
            if (active and e[cur][1]) or (nxt < len(e) and e[nxt][1]):
                isf = True
            if active:
                act.append((e, cur))
        if isf:
            vals = []
            for e, cur in act:
                x0, _, y0 = e[cur]
                if x0 == t:
                    vals.append(float(y0))
                else:
                    x1, _, y1 = e[cur + 1]
                    vals.append(float(y0) + (float(t - x0) * (float(y1) - float(y0))) / float(x1 - x0))
            r = agg_double(agg, vals)
            if r != r or math.isinf(r):
                raise ArithmeticError(len(out))
            out.append((t, False, r))
        else:
            vals = []
            for e, cur in act:
                x0, _, y0 = e[cur]
                if x0 == t:
                    vals.append(y0)
                else:
                    x1, _, y1 = e[cur + 1]
                    vals.append(wrap(y0 + jdiv(wrap((t - x0) * wrap(y1 - y0)), x1 - x0)))
            out.append((t, True, agg_long(agg, vals)))
    return out
