"""Series-sharded SpanGroups: the exchange path of
tsdbhip_spangroup_run (bounds / flags allreduce, grid-bitmap allgather + OR,
per-t partials allgather and rank-ordered combine) on a 1-rank RCCL
communicator (-m gpu; one GPU per box), and the shard plan plus the bench's
multi-process harness on CPU with gloo (world_size 2)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from helpers import I, F, T0, U32MAX, assert_same
import oracle
from opentsdb_amd import _abi, core, packing, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def sctx():
    from opentsdb_amd._lib import Context
    c = Context(0)
    c.comm_init(1, 0, Context.unique_id())
    yield c
    c.close()


def run_sharded(c, ss, **kw):
    start = kw.pop("start", 0)
    end = kw.pop("end", U32MAX)
    agg = kw.pop("agg", 0)
    g = core.run_spanset(c, ss, start, end, agg, sharded=True, **kw)
    o = oracle.spangroup(ss, start, end, agg, kw.get("rate", False), kw.get("ds_interval", 0), kw.get("ds_agg", 0))
    return g, o


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 1, 2, 3, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_sharded_regular_ds(sctx, agg, rate):
    ss = synth.regular(24, 2000, _abi.SYN_INT64_COUNTER, seed=7, step=10)
    g, o = run_sharded(sctx, ss, agg=agg, rate=rate, ds_interval=60, ds_agg=3)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 2, 4])
@pytest.mark.parametrize("rate", [False, True])
def test_sharded_regular_nods_direct(sctx, agg, rate):
    """no downsampling on regular series: the direct path (k_direct.hip), whose
    consecutive-rank test runs against the exchanged (global) grid"""
    ss = synth.regular(30, 1200, _abi.SYN_INT64_COUNTER, seed=5, step=5)
    g, o = run_sharded(sctx, ss, agg=agg, rate=rate)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 3, 4])
def test_sharded_c3s_shape(sctx, agg):
    ss = synth.regular(300, 3600, _abi.SYN_INT64_COUNTER, seed=3, step=1)
    g, o = run_sharded(sctx, ss, agg=agg, ds_interval=60, ds_agg=3)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 1, 2, 3, 4])
def test_sharded_many_chunks_combine(sctx, agg):
    """>= 64 reduce chunks per rank (2048 spans, T = 10 buckets): the rank's
    chunk partials go through k_combine_par (block per t, ordered tree)."""
    ss = synth.regular(2048, 600, _abi.SYN_INT64_COUNTER, seed=11, step=1)
    g, o = run_sharded(sctx, ss, agg=agg, ds_interval=60, ds_agg=3)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 2, 3])
@pytest.mark.parametrize("rate", [False, True])
def test_sharded_many_chunks_direct(sctx, agg, rate):
    """the direct path with >= 64 chunks per rank (1100 spans, T = 200)"""
    ss = synth.regular(1100, 200, _abi.SYN_INT64_COUNTER, seed=12, step=1)
    g, o = run_sharded(sctx, ss, agg=agg, rate=rate)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("agg", [0, 1, 3, 4])
@pytest.mark.parametrize("rate", [False, True])
@pytest.mark.parametrize("sharded", [False, True])
def test_many_chunks_large_t(sctx, agg, rate, sharded):
    """>= 64 chunks at T >= 1024 (1100 spans x 1200 points): the coalesced
    column merge (k_chunks_cols) as the finalize and as the rank combine"""
    ss = synth.regular(1100, 1200, _abi.SYN_INT64_COUNTER, seed=13, step=1)
    g = core.run_spanset(sctx, ss, 0, U32MAX, agg, sharded=sharded, rate=rate)
    o = oracle.spangroup(ss, 0, U32MAX, agg, rate, 0, 0)
    assert_same(g, o)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2])
@pytest.mark.parametrize("agg", [0, 2, 4])
def test_sharded_jittered_mixed(sctx, seed, agg):
    rng = np.random.default_rng(seed)
    spans = []
    for s in range(12):
        ts = T0 + 5 * s + np.cumsum(rng.integers(1, 400, 150))
        if s % 3 == 0:
            spans.append(F([(int(t), float(rng.integers(-40, 40)) / 4) for t in ts]))
        else:
            spans.append(I([(int(t), int(v)) for t, v in zip(ts, rng.integers(-10**6, 10**6, len(ts)))]))
    ss = packing.pack_spans(spans)
    for rate in (False, True):
        g, o = run_sharded(sctx, ss, agg=agg, rate=rate)
        assert_same(g, o)


@pytest.mark.gpu
def test_sharded_empty_span_error(sctx):
    """An error on one shard surfaces on every rank (exchanged before throwing)."""
    ss = packing.pack_spans([I([(T0 + 1, 1), (T0 + 2, 2)])])
    ss.span_row_start = np.array([0, 1, 1], np.uint64)  # second span has no rows
    g = core.run_spanset(sctx, ss, 0, U32MAX, 0, sharded=True)
    assert g[0] == _abi.E_EMPTY_SPAN


# ------------------------------------------------------------------- CPU ----
def shard_ranges(n_series, world):
    """bench.py's plan: contiguous span ranges, span order preserved."""
    return [(n_series * r // world, n_series * (r + 1) // world) for r in range(world)]


def test_shard_plan_covers_in_order():
    for n, w in [(1_000_000, 8), (7, 2), (3, 4), (100, 3)]:
        rs = shard_ranges(n, w)
        assert rs[0][0] == 0 and rs[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
        sizes = [b - a for a, b in rs]
        assert max(sizes) - min(sizes) <= 1


def _span_cells(ss, k):
    """(timestamps, value bytes) of span k of a SpanSet."""
    out_t, out_v = [], []
    for r in range(int(ss.span_row_start[k]), int(ss.span_row_start[k + 1])):
        n = int(ss.row_ncells[r])
        q = ss.qual_bytes[int(ss.row_qual_off[r]):int(ss.row_qual_off[r]) + 2 * n]
        out_t += [int(ss.row_base[r]) + ((int(q[2 * i]) << 8 | int(q[2 * i + 1])) >> 4) for i in range(n)]
        vo = int(ss.row_val_off[r])
        out_v.append(bytes(ss.val_bytes[vo:vo + int(ss.row_val_len[r])]))
    return out_t, b"".join(out_v)


def test_shards_hold_the_global_series():
    """A rank generating its span range (span0 = first global series) holds
    exactly those series of the unsharded group, so the ranks jointly hold
    the SpanGroup in TreeMap order."""
    whole = synth.regular(10, 700, _abi.SYN_INT64_COUNTER, seed=2, step=10)
    for a, b in shard_ranges(10, 3):
        part = synth.regular(b - a, 700, _abi.SYN_INT64_COUNTER, seed=2, step=10, span0=a)
        for k in range(b - a):
            assert _span_cells(part, k) == _span_cells(whole, a + k)


def test_sharded_aggregate_equals_whole_on_cpu():
    """Integer sum with aligned grids: per-shard oracle results added in rank
    order equal the whole group's (the combine the ranks perform)."""
    whole = synth.regular(9, 700, _abi.SYN_INT64_COUNTER, seed=4, step=10)
    o = oracle.spangroup(whole, 0, U32MAX, 0, False, 60, 3)
    acc = None
    for a, b in shard_ranges(9, 2):
        part = synth.regular(b - a, 700, _abi.SYN_INT64_COUNTER, seed=4, step=10, span0=a)
        p = oracle.spangroup(part, 0, U32MAX, 0, False, 60, 3)
        assert np.array_equal(p.ts, o.ts)
        acc = p.bits.copy() if acc is None else (acc.astype(np.uint64) + p.bits.astype(np.uint64)).astype(np.int64)
    assert np.array_equal(acc, o.bits)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_harness_gloo_world2():
    """bench.py's distributed harness (barrier, max-over-ranks timing, rank-0
    line) with world_size 2 over gloo on CPU, using its --dry-run step."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={env['MASTER_PORT']}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-run"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    import json
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["value"] > 0
    assert d["config"]["shards"] == [[0, 500000], [500000, 1000000]]


def test_bench_harness_groups_world2():
    """GROUP BY over 2 ranks: whole groups per rank (no exchange), group
    boundaries respected by the span split."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={env['MASTER_PORT']}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--dry-run",
           "--config", "c3s_gb100", "--groups", "3"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    import json
    d = json.loads(lines[0])
    assert d["config"]["shards"] == [[0, 333333], [333333, 1000000]]


def test_bench_rehearsal_split_and_single_line():
    """--rehearse-shards N at N=1 takes rank 0's 1/N shard, and the process's
    stdout holds the JSON line alone (native banners go to stderr)."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "2", "--warmup", "1", "--dry-run",
           "--rehearse-shards", "8"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = r.stdout.splitlines()
    assert len(lines) == 1, r.stdout
    import json
    d = json.loads(lines[0])
    assert d["n_gpus"] == 1 and len(d["config"]["shards"]) == 8
    assert d["config"]["shards"][0] == [0, 125000]


def test_bench_spawns_its_ranks_without_a_launcher():
    """`python bench.py --gpus 2` (no torchrun) starts 2 ranks itself and the
    line reports n_gpus 2; a WORLD_SIZE that disagrees with --gpus fails."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--dry-run"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    import json
    assert json.loads(lines[0])["n_gpus"] == 2
    r = subprocess.run(cmd, env=dict(env, WORLD_SIZE="1"), capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
