"""Pure-Python restatement of CompactionQueue.compact(row, compacted)
(src/core/CompactionQueue.java:243-743) — a second, independent restatement
used only to cross-check oracle/oracle.cc on random rows. Returns
(status, qualifier bytes, value bytes) with the row status codes of
include/tsdbhip.h; `decide` adds the flush path's write/delete decision
(:276, :355-404, :419-434) as (put?, KV index kept from the delete, or -1).
"""
NONE, SINGLE, TRIVIAL, COMPLEX, ERROR, OOB = 0, 1, 2, 3, 4, 5


class _Illegal(Exception):
    pass


class _Oob(Exception):
    pass


def _legacy(flags, value):  # floatingPointValueToFix :510-515
    return (flags & 0x8) != 0 and (flags & 0x7) == 0x3 and len(value) == 8


def _fixv(flags, value):  # fixFloatingPointValue :530-544
    if _legacy(flags, value):
        if value[:4] == b"\0\0\0\0":
            return value[4:]
        raise _Illegal()
    return value


def _fixq(flags, vlen):  # fixQualifierFlags :490-499 (byte arithmetic)
    return ((flags & ~0x7) | (vlen - 1)) & 0xFF


def _breakdown(row):  # breakDownValues :690-743
    cells = []
    for q, v in row:
        if len(q) == 2:
            av = _fixv(q[1], v)
            cells.append((bytes([q[0], _fixq(q[1], len(av))]), av))
            continue
        if len(v) == 0:
            raise _Oob()
        if v[-1] != 0:
            raise _Illegal()
        vi = 0
        for i in range(0, len(q), 2):
            vlen = (q[i + 1] & 0x7) + 1
            if vi + vlen > len(v):
                raise _Oob()
            cells.append((q[i:i + 2], v[vi:vi + vlen]))
            vi += vlen
        if vi != len(v) - 1:
            raise _Illegal()
    return cells


def _complex(row):  # complexCompact :600-679
    cells = sorted(_breakdown(row), key=lambda c: c[0])  # stable, unsigned bytes
    out_q, out_v = [], []
    last = -1
    prev = None
    for q, v in cells:
        delta = ((q[0] << 8) | q[1]) >> 4
        if delta == last:
            if q[1] != prev[0][1] or v != prev[1]:
                raise _Illegal()
            continue
        last, prev = delta, (q, v)
        out_q.append(q)
        out_v.append(v)
    return COMPLEX, b"".join(out_q), b"".join(out_v) + b"\0"


def compact(row):
    """row: list of (qualifier bytes, value bytes) in HBase order."""
    try:
        return _compact(list(row))
    except _Illegal:
        return ERROR, b"", b""
    except _Oob:
        return OOB, b"", b""


def _compact(row):
    if len(row) <= 1:
        if not row:
            return NONE, b"", b""
        q, v = row[0]
        if len(q) % 2 or not q:
            return NONE, b"", b""
        if len(q) == 2 and _legacy(q[1], v):
            nv = _fixv(q[1], v)
            return SINGLE, bytes([q[0], _fixq(q[1], len(nv))]), nv
        return SINGLE, q, v
    kept, trivial, last = [], True, -1
    for q, v in row:
        if len(q) != 2:
            if len(q) % 2 or not q:
                continue
            trivial = False
        else:
            delta = ((q[0] << 8) | q[1]) >> 4
            if delta <= last:
                raise _Illegal()
            last = delta
        kept.append((q, v))
    if len(kept) < 2:
        return _compact(kept)
    if trivial:  # trivialCompact :450-474
        qs, vs = [], []
        for q, v in kept:
            fv = _fixv(q[1], v)
            qs.append(bytes([q[0], _fixq(q[1], len(fv))]))
            vs.append(fv)
        return TRIVIAL, b"".join(qs), b"".join(vs) + b"\0"
    return _complex(kept)


def decide(row):
    """-> (status, qualifier, value, put, keep): compact() plus the flush
    path's writes for a row old enough to be written back. The KVs deleted
    are the row's even, non-empty qualifiers except index `keep`."""
    st, q, v = compact(row)
    if st == TRIVIAL:
        return st, q, v, True, -1   # the compacted qualifier is longer than any KV's
    if st != COMPLEX:
        return st, q, v, False, -1  # no put, no delete (returned early or threw)
    # `longest` (:283-312): row[0] as handed in, then every later valid
    # non-2-byte qualifier strictly longer than the current one
    li, ll = 0, len(row[0][0])
    for i, (kq, _) in enumerate(row):
        if len(kq) != 2 and len(kq) % 2 == 0 and kq and len(kq) > ll:
            li, ll = i, len(kq)
    if len(q) > ll:
        return st, q, v, True, -1
    dup = li if row[li][0] == q else next(
        (i for i, (kq, _) in enumerate(row) if kq and len(kq) % 2 == 0 and kq == q), -1)
    if dup < 0:
        return st, q, v, True, -1
    return st, q, v, row[dup][1] != v, dup
