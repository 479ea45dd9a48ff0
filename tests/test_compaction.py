"""CompactionQueue.compact (CompactionQueue.java:243-743): the oracle against
the reference's TestCompactionQueue vectors (test_oracle.py) and an
independent Python restatement on edge cases and random C5-style batches
(CPU), then the GPU path (tsdbhip_compact_rows) against the oracle,
byte-exact (-m gpu)."""
import struct

import numpy as np

import pytest


import closed_form_compaction as cfc
import oracle
from opentsdb_amd import _abi, compaction


def L(v):
    return struct.pack(">q", v)


def I4(v):
    return struct.pack(">i", v)


def Q(delta, flags):
    return struct.pack(">H", (delta << 4) | flags)


def compacted(cells):
    """trivialCompact layout of [(delta, flags, value)]."""
    return b"".join(Q(d, f) for d, f, _ in cells), b"".join(v for _, _, v in cells) + b"\0"


FB = struct.unpack(">I", struct.pack(">f", 4.2))[0]
LEGACY = b"\0\0\0\0" + struct.pack(">I", FB)


def edge_rows():
    c3 = compacted([(1, 7, L(4)), (2, 7, L(5)), (9, 3, I4(-2))])
    big = [(Q(d, 7), L(d * 3)) for d in range(3600)]
    bigc = compacted([(d, 7, L(d * 3)) for d in range(3600)])
    midc = compacted([(d, 7, L(d * 3)) for d in range(3000)])
    rows = {
        "empty": [],
        "junk only": [(b"\x01\x02\x03", b"xy")],
        "empty qualifier": [(b"", L(1))],
        "junk + single": [(b"\x01", b""), (Q(5, 7), L(9))],
        "two junk": [(b"\x01", b"a"), (b"\x01\x02\x03", b"b")],
        "single legacy ok": [(Q(3, 0xB), LEGACY)],
        "single legacy corrupt": [(Q(3, 0xB), b"\xff\xff\xff\xff" + LEGACY[4:])],
        "single compacted as-is": [(c3[0], c3[1])],
        "single compacted malformed": [(c3[0], b"\x01\x02")],
        "single long flagged 4": [(Q(3, 3), L(77))],
        "trivial zero-length value": [(Q(1, 7), b""), (Q(2, 7), L(1))],
        "trivial 9-byte value": [(Q(1, 7), b"123456789"), (Q(2, 7), L(1))],
        "trivial legacy": [(Q(1, 7), L(4)), (Q(2, 0xB), LEGACY), (Q(3, 0), b"\x05")],
        "trivial legacy corrupt": [(Q(1, 7), L(4)), (Q(2, 0xB), b"\0\0\0\1" + LEGACY[4:])],
        "trivial unsorted": [(Q(5, 7), L(4)), (Q(3, 7), L(5))],
        "trivial same delta": [(Q(5, 3), I4(4)), (Q(5, 7), L(5))],
        "trivial junk middle": [(Q(1, 0), b"\x01"), (b"\x09", b"zz"), (Q(2, 1), b"\x00\x02")],
        "trivial 3600": big,
        "complex dedupe": [(Q(1, 7), L(4)), (c3[0], c3[1]), (Q(5, 1), b"\x00\x07")],
        "complex unsorted singles": [(Q(5, 7), L(4)), (c3[0], c3[1]), (Q(4, 7), L(5))],
        "complex conflict value": [(Q(1, 7), L(99)), (c3[0], c3[1])],
        "complex conflict flags": [(Q(1, 3), I4(4)), (c3[0], c3[1])],
        "complex empty value": [(Q(0, 7), L(1)), (c3[0], b"")],
        "complex bad meta": [(Q(0, 7), L(1)), (c3[0], c3[1][:-1] + b"\x01")],
        "complex overflow": [(Q(0, 7), L(1)), (c3[0], c3[1][:10] + b"\0")],
        "complex extra bytes": [(Q(0, 7), L(1)), (c3[0], c3[1][:-1] + b"\x07\0")],
        "complex first error wins": [(Q(0, 0xB), b"\x01\0\0\0\0\0\0\0"), (c3[0], b"")],
        "complex oob before illegal": [(Q(0, 7), L(1)), (c3[0], b""), (c3[0] + Q(20, 7), b"\x01")],
        "complex internal dup": [(Q(0, 7), L(1)), compacted([(3, 0, b"\x01"), (3, 0, b"\x01")])],
        "complex legacy inside": [(Q(0, 7), L(1)), compacted([(3, 0xB, LEGACY), (4, 0, b"\x02")])],
        "complex legacy single": [(Q(0, 0xB), LEGACY), (c3[0], c3[1])],
        "complex 3000 + dups": [midc] + big[:3000],
        "complex 3600 + dups": [bigc] + big,
        "complex 3600 dup x2": [bigc, bigc] + big,
        "complex two compacted": [compacted([(1, 7, L(1)), (3, 7, L(3))]),
                                  compacted([(2, 7, L(2)), (4, 7, L(4))])],
        "complex junk": [(b"\x01", b"?"), (c3[0], c3[1]), (Q(10, 0), b"\x01")],
    }
    return rows


EDGE = edge_rows()


def check_against(res, expected):
    for r, (st, q, v) in enumerate(expected):
        assert res.row(r) == (st, q, v), (r, res.row(r)[0], st)


@pytest.mark.parametrize("name", list(EDGE))
def test_oracle_edge_rows(name):
    row = EDGE[name]
    res = oracle.compact_rows(compaction.pack_rows([row]))
    assert res.row(0) == cfc.compact(row)
    st, q, v, put, keep = cfc.decide(row)
    assert (bool(res.write[0]), int(res.keep_kv[0])) == (put, keep)


def test_oracle_decision_cases():
    """The write/delete decision (CompactionQueue.java:364-400) on rows
    built to reach each branch: the dup found as `longest`, found by the
    loop (a 2-byte KV equal to a deduplicated 1-cell compaction: same
    qualifier, value without the meta byte, so put but keep the cell), a junk row[0]
    longer than every valid qualifier (:283 takes it before :302 drops it)."""
    c12 = compacted([(1, 7, L(1)), (2, 7, L(2))])
    one = compacted([(3, 0, b"\x01"), (3, 0, b"\x01")])  # dedupes to the single cell (3, 0)
    rows = {
        "dup is longest, same value": ([(Q(1, 7), L(1)), c12, (Q(2, 7), L(2))], False, 1),
        "dup by loop, different value": ([(Q(3, 0), b"\x01"), one], True, 0),
        "junk row0 longest": ([(b"\x00\x01\x02\x03\x04", b"j"), c12, (Q(1, 7), L(1))], False, 1),
        "no dup": ([(Q(1, 7), L(1)), compacted([(2, 7, L(2)), (3, 7, L(3))])], True, -1),
    }
    b = compaction.pack_rows([r for r, _, _ in rows.values()])
    res = oracle.compact_rows(b)
    for i, (name, (row, put, keep)) in enumerate(rows.items()):
        assert res.row(i)[0] == cfc.COMPLEX, name
        assert (bool(res.write[i]), int(res.keep_kv[i])) == (put, keep), name
        assert cfc.decide(row)[3:] == (put, keep), name


def test_oracle_edge_statuses():
    """Hand-derived outcomes (CompactionQueue.java line refs in k_compact.hip)."""
    want = {"empty": cfc.NONE, "junk only": cfc.NONE, "two junk": cfc.NONE, "junk + single": cfc.SINGLE,
            "single legacy corrupt": cfc.ERROR, "single compacted malformed": cfc.SINGLE,
            "trivial unsorted": cfc.ERROR, "trivial same delta": cfc.ERROR,
            "trivial legacy corrupt": cfc.ERROR, "complex dedupe": cfc.COMPLEX,
            "complex unsorted singles": cfc.ERROR, "complex conflict value": cfc.ERROR,
            "complex conflict flags": cfc.ERROR, "complex empty value": cfc.OOB,
            "complex bad meta": cfc.ERROR, "complex overflow": cfc.OOB, "complex extra bytes": cfc.ERROR,
            "complex first error wins": cfc.ERROR, "complex oob before illegal": cfc.OOB,
            "complex 3000 + dups": cfc.COMPLEX, "complex 3600 + dups": cfc.COMPLEX,
            "complex 3600 dup x2": cfc.COMPLEX}
    res = oracle.compact_rows(compaction.pack_rows([EDGE[k] for k in want]))
    for r, (k, st) in enumerate(want.items()):
        assert res.row(r)[0] == st, k
    q, v = res.row(list(want).index("complex dedupe"))[1:]
    assert q == Q(1, 7) + Q(2, 7) + Q(5, 1) + Q(9, 3)
    assert v == L(4) + L(5) + b"\x00\x07" + I4(-2) + b"\0"


def test_oracle_random_batch_vs_restatement():
    b = compaction.synth_rows(3000, seed=11, p_complex=0.3, p_conflict=0.05, p_junk=0.05)
    res = oracle.compact_rows(b)
    rows = batch_rows(b)
    for r in range(b.n_rows):
        st, q, v, put, keep = cfc.decide(rows[r])
        assert res.row(r) == (st, q, v), r
        assert (bool(res.write[r]), int(res.keep_kv[r])) == (put, keep), r
    st = np.bincount(res.status, minlength=6)
    assert st[cfc.TRIVIAL] and st[cfc.COMPLEX] and st[cfc.ERROR] and st[cfc.SINGLE]


def batch_rows(b):
    """RowBatch -> list of rows of (qualifier, value) (test helper)."""
    rows = []
    for r in range(b.n_rows):
        qp, vp = int(b.row_qual_off[r]), int(b.row_val_off[r])
        row = []
        for k in range(int(b.row_kv_start[r]), int(b.row_kv_start[r + 1])):
            ql, vl = int(b.kv_qual_len[k]), int(b.kv_val_len[k])
            row.append((bytes(b.qual_bytes[qp:qp + ql]), bytes(b.val_bytes[vp:vp + vl])))
            qp += ql
            vp += vl
        rows.append(row)
    return rows


def test_synth_rows_shape():
    """C5 generator: HBase qualifier order, the advertised mix."""
    b = compaction.synth_rows(20000, seed=3)
    assert b.n_kvs > 20000 and b.row_qual_off[-1] == b.kv_qual_len.astype(np.int64).sum()
    rows = batch_rows(b)
    for row in rows[:2000]:
        qs = [q for q, _ in row]
        assert qs == sorted(qs)
    res = oracle.compact_rows(b)
    st = np.bincount(res.status, minlength=6)
    assert st[cfc.TRIVIAL] > 0.8 * b.n_rows
    assert 0.05 * b.n_rows < st[cfc.COMPLEX] < 0.12 * b.n_rows
    assert st[cfc.ERROR] > 0


def test_pack_rejects_long_kv():
    with pytest.raises(ValueError):
        compaction.pack_rows([[(Q(1, 7), b"x" * 70000)]])


# ------------------------------------------------------------------ GPU ----
def assert_same(g, o):
    assert np.array_equal(g.status, o.status)
    assert np.array_equal(g.qual_len, o.qual_len) and np.array_equal(g.val_len, o.val_len)
    assert np.array_equal(g.qual_off, o.qual_off) and np.array_equal(g.val_off, o.val_off)
    assert np.array_equal(g.packed_qual(), o.packed_qual())
    assert np.array_equal(g.packed_val(), o.packed_val())
    assert g.n_complex == o.n_complex
    assert np.array_equal(g.write, o.write), "row_write"
    assert np.array_equal(g.keep_kv, o.keep_kv), "row_keep_kv"


@pytest.mark.gpu
def test_gpu_compaction_golden(ctx):
    """TestCompactionQueue.java:77-299 vectors through the GPU."""
    import json
    import os
    gold = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "known_answers.json")))["compaction"]
    rows = [[(bytes.fromhex(q), bytes.fromhex(v)) for q, v in c["kvs"]] for c in gold]
    b = compaction.pack_rows(rows)
    g = compaction.compact_rows(ctx, b)
    assert_same(g, oracle.compact_rows(b))
    status = {"none": 0, "single": 1, "trivial": 2, "complex": 3, "error": 4}
    for r, c in enumerate(gold):
        st, q, v = g.row(r)
        assert st == status[c["status"]], c["name"]
        if "qual" in c:
            assert q.hex() == c["qual"] and v.hex() == c["val"], c["name"]
        assert g.decision(r, [len(k) for k, _ in rows[r]]) == (c["put"], c["delete"]), c["name"]


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(EDGE))
def test_gpu_compaction_edge(ctx, name):
    b = compaction.pack_rows([EDGE[name]])
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
def test_gpu_compaction_edge_batch(ctx):
    """All edge rows in one batch, twice, in two orders."""
    rows = list(EDGE.values())
    rows = rows + rows[::-1]
    b = compaction.pack_rows(rows)
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_gpu_compaction_random(ctx, seed):
    b = compaction.synth_rows(20000, seed=seed, p_complex=0.3, p_conflict=0.02, p_junk=0.02)
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
def test_gpu_compaction_long_rows(ctx):
    """Rows of up to 900 KVs (several waves of KVs per row)."""
    b = compaction.synth_rows(3000, seed=9, min_cells=300, max_cells=900, p_complex=0.5, p_conflict=0.01)
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
def test_gpu_compaction_rows_over_budget(ctx):
    """Rows of 2100-3000 KVs: each alone over k_compact_wave's and
    k_compact_rows' LDS budgets, next to short rows (pieces of one row, rows
    skipped)."""
    b = compaction.synth_rows(60, seed=11, min_cells=2100, max_cells=3000, p_complex=0.2, p_conflict=0.0)
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))
    rows = [[(Q(d, 7), L(d)) for d in range(n)] for n in (2, 2200, 3, 40, 2500, 2, 1)]
    b = compaction.pack_rows(rows)
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
def test_gpu_compaction_tiny_rows(ctx, seed):
    """Rows of 1-3 cells: many rows a 16-B chunk, piece edges inside rows' heads."""
    b = compaction.synth_rows(50000, seed=seed, min_cells=1, max_cells=3, p_complex=0.1, p_conflict=0.01)
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
def test_gpu_compaction_legacy_heavy(ctx):
    """Half the cells legacy 8-byte floats: rows with 0, 1, 2 and more holes
    (more than two go to the row kernel)."""
    kp = np.array([0.1, 0.1, 0.1, 0.1, 0.05, 0.05, 0.5, 0.0])
    for lo, hi in ((2, 4), (2, 40)):
        b = compaction.synth_rows(20000, seed=13, min_cells=lo, max_cells=hi, p_complex=0.05, kind_p=kp / kp.sum())
        assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
@pytest.mark.timeout(400)
def test_gpu_compaction_c5_full(ctx):
    """C5 at full size (1M rows, ~50M cells): bit-exact vs the oracle."""
    b = compaction.synth_rows(1_000_000, seed=5)
    assert_same(compaction.compact_rows(ctx, b), oracle.compact_rows(b))


@pytest.mark.gpu
def test_gpu_compaction_bad_offsets(ctx):
    b = compaction.pack_rows([[(Q(1, 7), L(1)), (Q(2, 7), L(2))]])
    b.row_val_off[1] += 1  # lengths no longer add up to the row's extent
    d = b.fill_desc(_abi.RowsDesc())
    res, out = compaction.out_buffers(b)
    import ctypes as C
    assert ctx._lib.tsdbhip_compact_rows(ctx.handle, C.byref(d), C.byref(out)) == _abi.E_INVALID_ARG


def _device_call(ctx, b, qcap=None, vcap=None):
    """tsdbhip_compact_rows with a device descriptor (HBM-resident rows and
    outputs, as bench.py's C5 line): the batch's extents are read by the
    kernels and checked at the call's end. -> (return code, RowsResult)"""
    import ctypes as C
    import torch
    dev = torch.device("cuda", 0)
    keep = []

    def up(a, ctype):
        t = torch.from_numpy(np.ascontiguousarray(a).view(np.uint8)).to(dev)
        keep.append(t)
        return C.cast(C.c_void_p(t.data_ptr()), C.POINTER(ctype))
    d = _abi.RowsDesc(flags=_abi.DESC_DEVICE, n_rows=b.n_rows, n_kvs=b.n_kvs,
                      row_kv_start=up(b.row_kv_start, C.c_uint64), row_qual_off=up(b.row_qual_off, C.c_uint64),
                      row_val_off=up(b.row_val_off, C.c_uint64), kv_qual_len=up(b.kv_qual_len, C.c_uint16),
                      kv_val_len=up(b.kv_val_len, C.c_uint16), qual_bytes=up(b.qual_bytes, C.c_uint8),
                      qual_nbytes=len(b.qual_bytes), val_bytes=up(b.val_bytes, C.c_uint8), val_nbytes=len(b.val_bytes))
    R = b.n_rows
    qcap = b.qual_extent + 64 if qcap is None else qcap
    vcap = b.val_extent + R + 64 if vcap is None else vcap
    o = {k: torch.zeros(max(n, 1), dtype=dt, device=dev) for k, n, dt in
         [("st", R, torch.uint8), ("qo", R, torch.int64), ("ql", R, torch.int32), ("vo", R, torch.int64),
          ("vl", R, torch.int32), ("q", qcap, torch.uint8), ("v", vcap, torch.uint8), ("w", R, torch.uint8),
          ("k", R, torch.int32)]}
    P = lambda t, ct: C.cast(C.c_void_p(t.data_ptr()), C.POINTER(ct))  # noqa: E731
    out = _abi.RowsOut(qual_capacity=qcap, val_capacity=vcap, row_status=P(o["st"], C.c_uint8),
                       row_qual_off=P(o["qo"], C.c_uint64), row_qual_len=P(o["ql"], C.c_uint32),
                       row_val_off=P(o["vo"], C.c_uint64), row_val_len=P(o["vl"], C.c_uint32),
                       qual_bytes=P(o["q"], C.c_uint8), val_bytes=P(o["v"], C.c_uint8),
                       row_write=P(o["w"], C.c_uint8), row_keep_kv=P(o["k"], C.c_int32))
    rc = ctx._lib.tsdbhip_compact_rows(ctx.handle, C.byref(d), C.byref(out))
    torch.cuda.synchronize()
    h = {k: v.cpu().numpy() for k, v in o.items()}
    res = compaction.RowsResult(h["st"][:R], h["qo"][:R].view(np.uint64), h["ql"][:R].view(np.uint32),
                                h["vo"][:R].view(np.uint64), h["vl"][:R].view(np.uint32), h["q"], h["v"],
                                h["w"][:R], h["k"][:R], int(out.n_complex))
    return rc, res, out


@pytest.mark.gpu
def test_gpu_compaction_device_desc(ctx):
    """HBM-resident rows and outputs (the bench's C5 call): same bytes and
    decisions as the oracle; qual_used / val_used from the kernels' extents"""
    b = compaction.synth_rows(20000, seed=17, p_complex=0.3, p_conflict=0.02, p_junk=0.02)
    rc, g, out = _device_call(ctx, b)
    assert rc == _abi.OK
    assert_same(g, oracle.compact_rows(b))
    assert out.qual_used == b.qual_extent and out.val_used == b.val_extent + b.n_rows


@pytest.mark.gpu
def test_gpu_compaction_device_desc_errors(ctx):
    """device descriptor: too small an output is E_CAPACITY, offsets past the
    buffers E_INVALID_ARG — found at the call's end, as the host descriptor
    finds them before it"""
    b = compaction.synth_rows(3000, seed=19)
    rc, _, _ = _device_call(ctx, b, qcap=b.qual_extent - 1)
    assert rc == _abi.E_CAPACITY
    rc, _, _ = _device_call(ctx, b, vcap=b.val_extent + b.n_rows - 1)
    assert rc == _abi.E_CAPACITY
    bad = compaction.RowBatch(b.row_kv_start.copy(), b.row_qual_off.copy(), b.row_val_off.copy(), b.kv_qual_len,
                              b.kv_val_len, b.qual_bytes, b.val_bytes)
    bad.row_qual_off[-1] = len(b.qual_bytes) + 16
    rc, _, _ = _device_call(ctx, bad)
    assert rc == _abi.E_INVALID_ARG
    rc, g, _ = _device_call(ctx, b)  # (the context is fine afterwards)
    assert rc == _abi.OK
    assert_same(g, oracle.compact_rows(b))
