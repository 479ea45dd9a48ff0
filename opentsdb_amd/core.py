"""Host-side mirror of the reference call surface for the aggregation path.

Mirrors (names, argument meaning, error behaviour):
  Aggregators / Aggregator        src/core/Aggregators.java:22-245, Aggregator.java:24-86
  Span (addRow)                   src/core/Span.java:33-132
  SpanGroup (ctor, add, size,
    aggregatedSize, iterator,
    timestamp/isInteger/
    longValue/doubleValue(i))     src/core/SpanGroup.java:46-254
  DataPoint                       src/core/DataPoint.java:20-56
  IllegalDataException            src/core/IllegalDataException.java
  group_by_and_aggregate          TsdbQuery.groupByAndAggregate (TsdbQuery.java:294-363),
                                  SpanCmp (TsdbQuery.java:594-621),
                                  Tags.getValueId (Tags.java:213-227)

The whole SpanGroup is evaluated by libtsdbhip on the GPU on first access
(tsdbhip_spangroup_run); iteration then replays the reference's lazy
exception behaviour: points before the failing one are delivered, then the
mapped exception is raised.
"""
import ctypes as C
import numpy as np

from . import _abi
from ._lib import Context, TsdbHipError
from .packing import KeyValue, SpanSet, pack_spans


class IllegalDataException(Exception):
    """net.opentsdb.core.IllegalDataException"""


class IllegalStateException(Exception):
    """java.lang.IllegalStateException ("Got NaN or Infinity")"""


class ArrayIndexOutOfBoundsException(IndexError):
    """java.lang.ArrayIndexOutOfBoundsException"""


def _exception_for(code, msg):
    if code == _abi.E_ILLEGAL_DATA:
        return IllegalDataException(msg)
    if code == _abi.E_NAN_INF:
        return IllegalStateException(msg)
    if code == _abi.E_EMPTY_SPAN:
        return AssertionError(msg)
    if code == _abi.E_OUT_OF_BOUNDS:
        return ArrayIndexOutOfBoundsException(msg)
    return TsdbHipError(code, msg)


class Aggregator:
    """One of the five stateless aggregators; identity = op code."""

    def __init__(self, name, code):
        self._name = name
        self.code = code

    def toString(self):
        return self._name

    __str__ = toString

    def __repr__(self):
        return f"Aggregator({self._name})"


class Aggregators:
    SUM = Aggregator("sum", _abi.AGG_SUM)
    MIN = Aggregator("min", _abi.AGG_MIN)
    MAX = Aggregator("max", _abi.AGG_MAX)
    AVG = Aggregator("avg", _abi.AGG_AVG)
    DEV = Aggregator("dev", _abi.AGG_DEV)
    _BY_NAME = {"sum": SUM, "min": MIN, "max": MAX, "avg": AVG, "dev": DEV}

    @classmethod
    def get(cls, name):
        try:
            return cls._BY_NAME[name]
        except KeyError:
            raise LookupError("No such aggregator: " + name) from None

    @classmethod
    def set(cls):
        return set(cls._BY_NAME)


class DataPoint:
    __slots__ = ("_ts", "_isint", "_bits")

    def __init__(self, ts, isint, bits):
        self._ts, self._isint, self._bits = int(ts), bool(isint), int(bits)

    def timestamp(self):
        return self._ts

    def isInteger(self):
        return self._isint

    def longValue(self):
        if not self._isint:
            raise TypeError("ClassCastException: value is a double")
        return self._bits

    def doubleValue(self):
        if self._isint:
            raise TypeError("ClassCastException: value is a long")
        return float(np.int64(self._bits).view(np.float64))

    def toDouble(self):
        return float(self._bits) if self._isint else self.doubleValue()

    def __repr__(self):
        v = self._bits if self._isint else self.doubleValue()
        return f"DataPoint({self._ts}, {v!r})"


class Span:
    """The compacted rows of one time series, in scan order. The row
    acceptance rules of Span.addRow are applied by the library."""

    def __init__(self, rows=None):
        self.rows = list(rows or [])

    def addRow(self, row: KeyValue):
        self.rows.append(row)


def run_spanset(ctx, spanset: SpanSet, start, end, agg, rate=False, ds_interval=0, ds_agg=0,
                exact=False, capacity=None, device_desc=None, sharded=False, span0=0, register_out=False):
    """Low-level: one tsdbhip_spangroup_run. Returns (code, ts, is_int, bits,
    n_input_points, err_index). sharded: this rank's shard of a group whose
    first span has global index span0. register_out: the result buffers
    registered (tsdbhip_host_register, as the JNI bridge registers its
    DirectByteBuffers) for the call."""
    desc = _abi.SgDesc()
    if device_desc is not None:
        C.pointer(desc)[0] = device_desc
    else:
        spanset.fill_desc(desc)
        desc.flags = 0
    desc.start_time, desc.end_time = int(start), int(end)
    desc.rate, desc.agg, desc.ds_agg = int(bool(rate)), int(agg), int(ds_agg)
    desc.ds_interval = int(ds_interval)
    if exact:
        desc.flags |= _abi.EXACT_ORDER
    if sharded:  # this rank's shard; exchange over the ctx communicator
        desc.flags |= _abi.SHARDED
        desc.span0 = int(span0)
    cap = capacity
    if cap is None:
        cap = max(1, spanset.n_cells()) if spanset is not None else 1 << 20
    ts = np.zeros(cap, np.int64)
    isi = np.zeros(cap, np.uint8)
    bits = np.zeros(cap, np.int64)
    out = _abi.SgOut()
    out.capacity = cap
    out.ts = _abi.ptr(ts, C.c_int64)
    out.is_int = _abi.ptr(isi, C.c_uint8)
    out.bits = _abi.ptr(bits, C.c_int64)
    regs = []
    try:
        if register_out:
            for a in (ts, isi, bits):
                ctx.check(ctx._lib.tsdbhip_host_register(ctx.handle, a.ctypes.data_as(C.c_void_p), a.nbytes))
                regs.append(a)
        rc = ctx._lib.tsdbhip_spangroup_run(ctx.handle, C.byref(desc), C.byref(out))
    finally:
        for a in regs:
            ctx._lib.tsdbhip_host_unregister(ctx.handle, a.ctypes.data_as(C.c_void_p))
    n = int(out.n_out)
    return rc, ts[:n], isi[:n], bits[:n], int(out.n_input_points), int(out.err_index)


def run_spanset_batch(ctx, spanset: SpanSet, group_span_start, start, end, agg, rate=False, ds_interval=0,
                      ds_agg=0, exact=False, capacities=None, device_desc=None):
    """Low-level: one tsdbhip_spangroup_run_batch over the groups
    [gss[g], gss[g+1]) of spanset. Returns (code, [per-group tuples as
    run_spanset returns them])."""
    gss = np.ascontiguousarray(group_span_start, np.uint32)
    G = len(gss) - 1
    desc = _abi.SgDesc()
    if device_desc is not None:
        C.pointer(desc)[0] = device_desc
    else:
        spanset.fill_desc(desc)
        desc.flags = 0
    desc.start_time, desc.end_time = int(start), int(end)
    desc.rate, desc.agg, desc.ds_agg = int(bool(rate)), int(agg), int(ds_agg)
    desc.ds_interval = int(ds_interval)
    if exact:
        desc.flags |= _abi.EXACT_ORDER
    if capacities is None:
        cells = np.concatenate([[0], np.cumsum(spanset.row_ncells.astype(np.int64))])
        srs = spanset.span_row_start.astype(np.int64)
        cum = cells[srs]  # cells before span s
        capacities = np.maximum(1, cum[gss[1:].astype(np.int64)] - cum[gss[:-1].astype(np.int64)])
    outs = (_abi.SgOut * max(G, 1))()
    bufs = []
    for g in range(G):
        cap = int(capacities[g])
        ts, isi, bits = np.zeros(cap, np.int64), np.zeros(cap, np.uint8), np.zeros(cap, np.int64)
        bufs.append((ts, isi, bits))
        outs[g].capacity = cap
        outs[g].ts = _abi.ptr(ts, C.c_int64)
        outs[g].is_int = _abi.ptr(isi, C.c_uint8)
        outs[g].bits = _abi.ptr(bits, C.c_int64)
    rc = ctx._lib.tsdbhip_spangroup_run_batch(ctx.handle, C.byref(desc), G, _abi.ptr(gss, C.c_uint32), outs)
    res = []
    for g in range(G):
        n = int(outs[g].n_out)
        ts, isi, bits = bufs[g]
        res.append((int(outs[g].err_code), ts[:n], isi[:n], bits[:n], int(outs[g].n_input_points),
                    int(outs[g].err_index)))
    return rc, res


class SpanGroup:
    """net.opentsdb.core.SpanGroup over libtsdbhip (SpanGroup.java:104-254)."""

    _default_ctx = None

    def __init__(self, tsdb, start_time, end_time, spans, rate, aggregator, interval=0,
                 downsampler=None, ctx=None):
        self.start_time = int(start_time)
        self.end_time = int(end_time)
        self.spans = []
        self.rate = bool(rate)
        self.aggregator = aggregator
        self.sample_interval = int(interval)
        self.downsampler = downsampler
        self._ctx = ctx
        self._result = None
        if spans is not None:
            for s in spans:
                self.add(s)

    def add(self, span):
        # SpanGroup.add's time filter (SpanGroup.java:135-139) needs the
        # assembled span; the library applies it, so every span is handed over.
        self.spans.append(span)
        self._result = None

    def _context(self):
        if self._ctx is None:
            if SpanGroup._default_ctx is None:
                SpanGroup._default_ctx = Context(0)
            self._ctx = SpanGroup._default_ctx
        return self._ctx

    def _run(self):
        if self._result is None:
            ss = pack_spans([s.rows for s in self.spans])
            ds = self.downsampler is not None and self.sample_interval > 0
            self._result = run_spanset(self._context(), ss, self.start_time, self.end_time,
                                       self.aggregator.code, self.rate,
                                       self.sample_interval if ds else 0,
                                       self.downsampler.code if ds else 0)
        return self._result

    def _points(self):
        rc, ts, isi, bits, _, _ = self._run()
        for i in range(len(ts)):
            yield DataPoint(ts[i], isi[i], bits[i])
        if rc:
            raise _exception_for(rc, self._context().last_error())

    def aggregatedSize(self):
        return self._run()[4]

    def size(self):
        n = 0
        for _ in self._points():
            n += 1
        return n

    def iterator(self):
        return self._points()

    __iter__ = iterator

    def _get(self, i):
        if i < 0:
            raise IndexError("negative index: %d" % i)
        for j, dp in enumerate(self._points()):
            if j == i:
                return dp
        raise IndexError("index %d too large" % i)

    def timestamp(self, i):
        return self._get(i).timestamp()

    def isInteger(self, i):
        return self._get(i).isInteger()

    def longValue(self, i):
        return self._get(i).longValue()

    def doubleValue(self, i):
        return self._get(i).doubleValue()


# ---------------------------------------------------------------- GROUP BY ----
def span_cmp_key(row_key, metric_width=3):
    """Sort key equivalent to TsdbQuery.SpanCmp (TsdbQuery.java:594-621):
    metric id, then the tags, skipping the 4-byte base time; unsigned bytes,
    a shorter key first on a common prefix (Python bytes order)."""
    return bytes(row_key[:metric_width]) + bytes(row_key[metric_width + 4:])


def get_value_id(row_key, tag_id, metric_width=3, name_width=3, value_width=3):
    """Tags.getValueId (Tags.java:213-227): the value id of tag `tag_id` in
    the row key, or None."""
    pos = metric_width + 4
    while pos < len(row_key):
        if bytes(row_key[pos:pos + name_width]) == bytes(tag_id):
            pos += name_width
            return bytes(row_key[pos:pos + value_width])
        pos += name_width + value_width
    return None


def plan_groups(row_keys, group_bys, metric_width=3, name_width=3, value_width=3):
    """The grouping of TsdbQuery.groupByAndAggregate (TsdbQuery.java:294-363)
    as a plan: row_keys are the spans' row keys (any order, one per span).
    Returns (group_keys, order, group_span_start): the span indices in batch
    order (ByteMap order of the group keys, then SpanCmp order within a
    group) and the group boundaries. Spans without every group_by tag are
    dropped, as the reference does (with its log line)."""
    idx = sorted(range(len(row_keys)), key=lambda i: span_cmp_key(row_keys[i], metric_width))
    if group_bys is None:
        return [b""], idx, [0, len(idx)]
    tag_ids = sorted(bytes(t) for t in group_bys)  # group_bys is sorted by id
    groups = {}
    for i in idx:
        parts = []
        for t in tag_ids:
            v = get_value_id(row_keys[i], t, metric_width, name_width, value_width)
            if v is None:
                parts = None
                break
            parts.append(v)
        if parts is None:
            continue  # "WTF? Dropping span for row ..." (TsdbQuery.java:339-344)
        groups.setdefault(b"".join(parts), []).append(i)
    keys = sorted(groups)  # ByteMap: unsigned lexicographic
    order, gss = [], [0]
    for k in keys:
        order.extend(groups[k])
        gss.append(len(order))
    return keys, order, gss


def group_by_and_aggregate(spans, group_bys, start_time, end_time, rate, aggregator, interval=0,
                           downsampler=None, ctx=None, metric_width=3, name_width=3, value_width=3):
    """TsdbQuery.groupByAndAggregate over libtsdbhip: `spans` maps row key
    bytes -> Span (findSpans' TreeMap), `group_bys` the tag-name ids to group
    by (None: one group). Returns the SpanGroups in the reference's order,
    all evaluated by one tsdbhip_spangroup_run_batch; each raises its own
    exception lazily while iterated, like the reference's."""
    keys = list(spans)
    if not keys:
        return []
    gkeys, order, gss = plan_groups(keys, group_bys, metric_width, name_width, value_width)
    groups = [SpanGroup(None, start_time, end_time, [spans[keys[i]] for i in order[gss[g]:gss[g + 1]]], rate,
                        aggregator, interval, downsampler, ctx) for g in range(len(gkeys))]
    if not groups:
        return []
    ss = pack_spans([spans[keys[i]].rows for i in order])
    ds = downsampler is not None and interval > 0
    c = groups[0]._context()
    _, res = run_spanset_batch(c, ss, gss, start_time, end_time, aggregator.code, rate,
                               interval if ds else 0, downsampler.code if ds else 0)
    for grp, r in zip(groups, res):
        grp._ctx = c
        grp._result = r
    return groups


# ------------------------------------------------------------ output text ----
FMT_ASCII, FMT_GNUPLOT, FMT_CLI = 0, 1, 2


def format_points(mode, ts, is_int, bits, metric="", tags="", utc_offset=0):
    """tsdbhip_format_points: the lines GraphHandler.respondAsciiQuery
    (GraphHandler.java:785-808), Plot.dumpToFiles (Plot.java:190-204) or
    CliQuery (CliQuery.java:161-170) print for these points. Raises
    IllegalStateException on a NaN/Infinity where the reference does."""
    from ._lib import lib
    L = lib()
    ts = np.ascontiguousarray(ts, np.int64)
    isi = np.ascontiguousarray(is_int, np.uint8)
    bits = np.ascontiguousarray(bits, np.int64)
    n = len(ts)
    cap = max(64, n * (len(metric) + len(tags) + 64))
    buf = C.create_string_buffer(cap)
    rc = L.tsdbhip_format_points(mode, metric.encode(), tags.encode(), int(utc_offset), _abi.ptr(ts, C.c_int64),
                                 _abi.ptr(isi, C.c_uint8), _abi.ptr(bits, C.c_int64), n, buf, cap)
    if rc == _abi.E_NAN_INF:
        raise IllegalStateException("NaN or Infinity")
    if rc < 0:
        raise TsdbHipError(int(rc), "tsdbhip_format_points")
    return buf.raw[:rc].decode()
