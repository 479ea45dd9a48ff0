#!/usr/bin/env python3
"""Benchmark of the query-time aggregation hot path on MI355X.

Metric (BASELINE.json): input data points/sec aggregated (node) + % HBM
roofline. A step is one tsdbhip_spangroup_run over one HBM-resident SpanGroup
(the row bytes of TsdbQuery.findSpans, generated on the device): span
assembly, RowSeq decode, greedy downsampling, union grid, lerp/rate merge,
aggregation, and the RCCL exchange when sharded.

Default workload (N=1..8, strong scaling): C3* — 1M series x 3600 points
@1s, 8-byte long counters (IncomingDataPoints encoding), sum aggregator with
1m-avg downsampling (the north-star target configuration); series sharded
over the ranks by contiguous span ranges. `--config c2` runs configs[1]
(10k float series x 1 day @10s, avg + 1m-avg).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3s|c2|c1]
       (N>1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from opentsdb_amd import _abi, synth  # noqa: E402
from opentsdb_amd._lib import Context, lib  # noqa: E402

METRIC = "input data points/sec aggregated (node) + % HBM roofline, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec

def _cfg(n_series, n_points, step, kind, agg, dsi=0, dsa=0, rate=False, gen="device", desc="", groups=1):
    return dict(n_series=n_series, n_points=n_points, step=step, kind=kind, agg=agg, dsi=dsi, dsa=dsa,
                rate=rate, gen=gen, desc=desc, groups=groups)


I64, F32 = _abi.SYN_INT64_COUNTER, _abi.SYN_FLOAT32
SUM, MIN, MAX, AVG, DEV = _abi.AGG_SUM, _abi.AGG_MIN, _abi.AGG_MAX, _abi.AGG_AVG, _abi.AGG_DEV
CONFIGS = {
    # BASELINE.json configs; the default line is c3s (the north-star target)
    "c3s": _cfg(1_000_000, 3600, 1, I64, SUM, 60, AVG,
                desc="C3*: 1M series x 3600 pts @1s (3.6G pts), int64 counters, sum + 1m-avg downsample"),
    "c1": _cfg(100, 3600, 1, I64, SUM, desc="C1: 100 int series x 3600 pts @1s, sum, no downsample"),
    "c2": _cfg(10_000, 8640, 10, F32, AVG, 60, AVG,
               desc="C2: 10k float32 series x 1 day @10s (86.4M pts), avg + 1m-avg downsample"),
    "c3": _cfg(1_000_000, 3600, 1, I64, SUM, desc="C3 (sum, no rate): 1M series x 3600 pts @1s, int64 counters"),
    "c3r_sum": _cfg(1_000_000, 3600, 1, I64, SUM, rate=True, desc="C3: 1M series x 3600 pts @1s, rate, sum"),
    "c3r_max": _cfg(1_000_000, 3600, 1, I64, MAX, rate=True, desc="C3: 1M series x 3600 pts @1s, rate, max"),
    "c3r_dev": _cfg(1_000_000, 3600, 1, I64, DEV, rate=True, desc="C3: 1M series x 3600 pts @1s, rate, dev"),
    "c3_dev": _cfg(1_000_000, 3600, 1, I64, DEV,
                   desc="C3: 1M series x 3600 pts @1s, integer dev (no rate: the reference's sequential Welford)"),
    "c3_dev_100k": _cfg(100_000, 3600, 1, I64, DEV, desc="C3 shape, 100k series, integer dev (no rate)"),
    "c4": _cfg(1000, 11500, 0, -1, SUM, gen="jitter",
               desc="C4: 1000 jittered series (gaps U{1..6960}s, ~11.5k pts each, 50% float32 series, "
                    "1% float cells), ~10M-point union grid, sum"),
    "c4i": _cfg(1000, 11500, 0, -1, SUM, gen="jitter_int",
                desc="C4-int: the C4 timestamps with all-int series (the int64 lerp path), sum"),
    # GROUP BY: the C3* spans as the SpanGroup[] of
    # TsdbQuery.groupByAndAggregate, all groups in one tsdbhip_spangroup_run_batch
    "c3s_gb100": _cfg(1_000_000, 3600, 1, I64, SUM, 60, AVG, groups=100,
                      desc="C3* GROUP BY host=* (100 groups x 10k series), sum + 1m-avg downsample"),
    "c3s_gb10k": _cfg(1_000_000, 3600, 1, I64, SUM, 60, AVG, groups=10_000,
                      desc="C3* GROUP BY host=* (10k groups x 100 series), sum + 1m-avg downsample"),
    "c3_gb100": _cfg(1_000_000, 3600, 1, I64, SUM, groups=100,
                     desc="C3 GROUP BY host=* (100 groups x 10k series), sum, no downsample"),
    # secondary path (configs[4]): row compaction, see bench_c5
    "c5": _cfg(1_000_000, 0, 0, 0, 0, gen="rows",
               desc="C5: row compaction, 1M rows / ~48M raw cells (1..99 per row, mixed widths, legacy floats, "
                    "10% pre-compacted rows with late singles + exact dups, 0.1% conflicting dups)"),
}


def host_spanset(cfg, lo, hi, seed=4):
    """Host-generated SpanGroup of a config (the jittered C4 shapes), spans [lo, hi)."""
    ff = 0.5 if cfg["gen"] == "jitter" else 0.0
    fc = 0.01 if cfg["gen"] == "jitter" else 0.0
    ss = synth.jittered_packed(cfg["n_series"], cfg["n_points"], seed=seed, float_frac=ff, float_cell_frac=fc)
    if (lo, hi) == (0, cfg["n_series"]):
        return ss
    r0, r1 = int(ss.span_row_start[lo]), int(ss.span_row_start[hi])
    from opentsdb_amd.packing import SpanSet
    return SpanSet((ss.span_row_start[lo:hi + 1] - r0).astype(np.uint64), ss.row_base[r0:r1],
                   ss.row_ncells[r0:r1], ss.row_qual_off[r0:r1], ss.row_val_off[r0:r1], ss.row_val_len[r0:r1],
                   ss.qual_bytes, ss.val_bytes)


def spanset_row_bytes(ss):
    """SURVEY.md §8(d) algorithmic input bytes of a SpanSet's rows."""
    n = ss.row_ncells.astype(np.int64)
    return int((4 + 2 * n + ss.row_val_len.astype(np.int64)).sum())


def ref_row_bytes(n_series, n_points, step, kind):
    """per row 4 B base_time + 2 B/cell + value bytes + meta byte."""
    k = 3600 // step
    w = 4 if kind == _abi.SYN_FLOAT32 else 8
    full, rem = divmod(n_points, k)
    per_span = full * (4 + 2 * k + k * w + (1 if k > 1 else 0))
    if rem:
        per_span += 4 + 2 * rem + rem * w + (1 if rem > 1 else 0)
    return n_series * per_span


def kbase(name):
    """a profiled kernel's base name: template arguments and the occupancy
    variant's suffix dropped (k_reduce_w4<0, 2, ...> -> k_reduce)"""
    b = name.split("<")[0]
    return b[:-3] if b.endswith("_w4") else b


def pmc_traffic(config, kernel, world):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC
    summary of this config (profiles/pmc_<config>.json, made by
    profiles/profile.sh + pmc_summary.py: 2 x FETCH_SIZE + WRITE_SIZE)."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if world != 1 or not os.path.exists(path):
        return None, None
    ks = json.load(open(path)).get("kernels", {})
    # every instantiation of the kernel launches once per step (e.g. the
    # integer and float k_ds_spans), and the timed region covers them all
    names = kernel.split("+")  # (a "+"-joined name: the kernels the timed bracket covers)
    tot = sum(e["hbm_bytes_per_launch"] for name, e in ks.items()
              if kbase(name) in names and e.get("hbm_bytes_per_launch"))
    return (tot, os.path.relpath(path, ROOT)) if tot else (None, None)


# VALU issue peak: a wave64 VALU instruction takes 2 cycles of its SIMD
# (MI355X_MICROARCH.md §SIMD); 256 CUs x 4 SIMDs at 2.4 GHz.
VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2


def pmc_valu(config, kernel):
    """VALU wave-instructions per launch of `kernel` (SQ_INSTS_VALU) from the
    committed PMC summary of this config, or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None, None
    ks = json.load(open(path)).get("kernels", {})
    tot = sum(e.get("valu_insts_per_launch") or 0 for name, e in ks.items() if kbase(name) == kernel)
    return (tot, os.path.relpath(path, ROOT)) if tot else (None, None)


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return None, 0, 1, int(os.environ.get("LOCAL_RANK", "0"))
    import torch.distributed as dist
    dist.init_process_group("gloo")
    return dist, dist.get_rank(), dist.get_world_size(), int(os.environ.get("LOCAL_RANK", "0"))


def host_threads():
    """P = the cores this process may actually use (SURVEY.md §8(d):
    independent SpanGroups on nproc threads, TsdbQuery.java:322-362): the
    affinity set, capped by the cgroup's CPU quota (the GPU box shows the
    whole machine's cores in its affinity mask but grants a share of them;
    more threads than granted CPUs only time-slice)."""
    try:
        n = max(1, len(os.sched_getaffinity(0)))
    except AttributeError:
        n = max(1, os.cpu_count() or 1)
    q = cpu_quota()
    return max(1, min(n, int(q))) if q else n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_quota():
    """CPUs the cgroup grants this process (cpu.max), or None when unlimited:
    the GPU box shows the whole machine's cores but may grant a share."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1.0, int(q) / int(per))
    except (OSError, ValueError):
        return None


def run_pool(fn, probe, seconds):
    """Runs fn() (one independent unit: a SpanGroup or a row batch) on
    host_threads() threads pulling from one work counter, sized so the run
    takes ~`seconds` wall time. Returns (units done, wall seconds, threads,
    granted CPUs, CPU seconds the threads consumed). CPU seconds ~ threads x
    wall means the threads ran the whole time; per-unit CPU time above the
    1-thread probe then measures contention for the shared memory system."""
    threads = host_threads()
    quota = cpu_quota()
    total = max(threads, int(seconds * threads / max(probe, 1e-4)))
    left = [total]
    cpu = [0.0] * threads
    lock = threading.Lock()

    def work(i):
        c0 = time.thread_time()
        while True:
            with lock:
                if left[0] <= 0:
                    break
                left[0] -= 1
            fn()
        cpu[i] = time.thread_time() - c0

    ths = [threading.Thread(target=work, args=(i,)) for i in range(threads)]
    t = time.perf_counter()
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return total, time.perf_counter() - t, threads, quota, sum(cpu)


def pool_note(n, wall, threads, cpu_s, probe):
    """What limited the P-thread run: parallel efficiency against the 1-thread
    probe, and whether the threads were on a CPU (cpu_s / (threads x wall))
    or each unit simply took longer (cpu per unit / probe: shared caches and
    DRAM bandwidth)."""
    eff = (n * probe / wall) / threads
    busy = cpu_s / max(threads * wall, 1e-9)
    slow = (cpu_s / max(n, 1)) / max(probe, 1e-9)
    return (f"parallel efficiency {eff:.2f} of {threads} x 1-thread; threads on CPU {busy:.0%} of the wall time; "
            f"CPU time per unit {slow:.2f}x the 1-thread probe")


def cpu_baseline(cfg_name, seconds=10.0):
    """The oracle (C++ restatement of the reference's Java iterators) on the
    host cores: independent SpanGroups on P = nproc threads (group-by style,
    TsdbQuery.java:322-362); a bounded sample of the same workload shape."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    cfg = CONFIGS[cfg_name]
    if cfg["gen"] == "device":
        n_points = cfg["n_points"]
        sample_series = max(1, min(cfg["n_series"], 200_000 // max(1, n_points // 100)))
        ss = synth.regular(sample_series, n_points, cfg["kind"], seed=1, step=cfg["step"])
        what = f"{sample_series} series x {n_points} pts of the same workload"
        cap = n_points if not cfg["dsi"] else n_points * cfg["step"] // cfg["dsi"] + 2
    else:
        sample_series = 20
        ss = host_spanset(dict(cfg, n_series=sample_series), 0, sample_series, seed=11)
        what = f"{sample_series} series of the same generator (~{cfg['n_points']} pts each)"
        cap = ss.n_cells() + 16
    args = (0, (1 << 32) - 1, cfg["agg"], cfg["rate"], cfg["dsi"], cfg["dsa"])
    oracle.lib()
    # probe one run, then size the sample to ~`seconds` of wall time
    t = time.perf_counter()
    r = oracle.spangroup(ss, *args, capacity=cap)
    probe = time.perf_counter() - t
    n, wall, threads, quota, cpu_s = run_pool(lambda: oracle.spangroup(ss, *args, capacity=cap), probe, seconds)
    return {
        "value": n * r.n_input_points / wall, "unit": "input points/s", "cores": threads, "kind": "port",
        "cpu_model": cpu_model(), "cgroup_cpus": quota,
        "value_1core": r.n_input_points / probe,
        "sample": f"{what}, {n} SpanGroups on {threads} threads, {wall:.1f} s wall; "
                  f"{pool_note(n, wall, threads, cpu_s, probe)} "
                  f"(oracle/oracle.cc: C++ restatement of SpanGroup/Span/RowSeq/Aggregators; "
                  f"no JVM in the image)",
    }


def cpu_baseline_c5(batch, seconds=10.0):
    """oracle_compact_rows (C++ restatement of CompactionQueue.compact) on
    the host cores: independent row batches on P = nproc threads, a bounded
    sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from opentsdb_amd import compaction
    rows = min(batch.n_rows, 20000)
    k1 = int(batch.row_kv_start[rows])
    sub = compaction.RowBatch(batch.row_kv_start[:rows + 1].copy(), batch.row_qual_off[:rows + 1].copy(),
                              batch.row_val_off[:rows + 1].copy(), batch.kv_qual_len[:k1].copy(),
                              batch.kv_val_len[:k1].copy(), batch.qual_bytes, batch.val_bytes)
    cells = int(sub.kv_qual_len.astype(np.int64).sum() // 2)  # raw cells (2 qualifier bytes each)
    t = time.perf_counter()
    oracle.compact_rows(sub)
    probe = time.perf_counter() - t
    n, wall, threads, quota, cpu_s = run_pool(lambda: oracle.compact_rows(sub), probe, seconds)
    return {"value": n * cells / wall, "unit": "raw cells/s", "cores": threads, "kind": "port",
            "cpu_model": cpu_model(), "cgroup_cpus": quota,
            "value_1core": cells / probe,
            "sample": f"first {rows} rows ({cells} cells) of the same batch, {n} batches on {threads} threads, "
                      f"{wall:.1f} s wall; {pool_note(n, wall, threads, cpu_s, probe)} "
                      f"(oracle/oracle.cc: C++ restatement of CompactionQueue.compact; no JVM in the image)"}


_JSON_OUT = None


def set_options(ctx, opts):
    for o in opts:
        name, _, value = o.partition("=")
        ctx.set_option(name, value)


def emit(res):
    """The one JSON line, on the process's original stdout. main() points fd 1
    at stderr first, so banners native libraries print to stdout (RCCL's
    version block at communicator init) cannot land beside the line."""
    out = _JSON_OUT or sys.stdout
    print(json.dumps(res), file=out, flush=True)


# every kernel tsdbhip_compact_rows launches (the C5 line's traffic is their
# sum per call, from the committed PMC summary)
C5_KERNELS = ("k_compact_wave", "k_compact_rows", "k_compact_complex", "k_compact_dups")


def bench_c5(args):
    """C5 (configs[4]): tsdbhip_compact_rows over 1M HBM-resident rows."""
    import torch
    from opentsdb_amd import compaction
    t0 = time.perf_counter()
    mix = {}
    if args.c5_mix == "plain":  # no row needs a fix: trivialCompact is a copy
        mix = dict(p_complex=0.0, p_conflict=0.0, p_junk=0.0,
                   kind_p=np.array([0.25, 0.2, 0.2, 0.2, 0.1, 0.05, 0.0, 0.0]))
    elif args.c5_mix == "nocomplex":
        mix = dict(p_complex=0.0, p_conflict=0.0)
    b = compaction.synth_rows(args.series or 1_000_000, seed=5, **mix)
    gen_s = time.perf_counter() - t0
    ctx = Context(0)
    set_options(ctx, args.option)
    L = lib()
    dev = torch.device("cuda", 0)
    keep = []

    def up(a, ctype):
        t = torch.from_numpy(a.view(np.uint8)).to(dev)
        keep.append(t)
        return C.cast(C.c_void_p(t.data_ptr()), C.POINTER(ctype))

    d = _abi.RowsDesc(flags=_abi.DESC_DEVICE, n_rows=b.n_rows, n_kvs=b.n_kvs,
                      row_kv_start=up(b.row_kv_start, C.c_uint64), row_qual_off=up(b.row_qual_off, C.c_uint64),
                      row_val_off=up(b.row_val_off, C.c_uint64), kv_qual_len=up(b.kv_qual_len, C.c_uint16),
                      kv_val_len=up(b.kv_val_len, C.c_uint16), qual_bytes=up(b.qual_bytes, C.c_uint8),
                      qual_nbytes=len(b.qual_bytes), val_bytes=up(b.val_bytes, C.c_uint8),
                      val_nbytes=len(b.val_bytes))
    R = b.n_rows
    qcap, vcap = b.qual_extent + 64, b.val_extent + R + 64
    o = {k: torch.zeros(n, dtype=dt, device=dev) for k, n, dt in
         [("st", R, torch.uint8), ("qo", R, torch.int64), ("ql", R, torch.int32), ("vo", R, torch.int64),
          ("vl", R, torch.int32), ("q", qcap, torch.uint8), ("v", vcap, torch.uint8), ("w", R, torch.uint8),
          ("k", R, torch.int32)]}
    P = lambda t, ct: C.cast(C.c_void_p(t.data_ptr()), C.POINTER(ct))  # noqa: E731
    out = _abi.RowsOut(qual_capacity=qcap, val_capacity=vcap, row_status=P(o["st"], C.c_uint8),
                       row_qual_off=P(o["qo"], C.c_uint64), row_qual_len=P(o["ql"], C.c_uint32),
                       row_val_off=P(o["vo"], C.c_uint64), row_val_len=P(o["vl"], C.c_uint32),
                       qual_bytes=P(o["q"], C.c_uint8), val_bytes=P(o["v"], C.c_uint8),
                       row_write=P(o["w"], C.c_uint8), row_keep_kv=P(o["k"], C.c_int32))

    def step_once():
        ctx.check(L.tsdbhip_compact_rows(ctx.handle, C.byref(d), C.byref(out)))

    for _ in range(args.warmup):
        step_once()
    ctx.timing_totals(reset=True)  # (per-call HIP-event timings, summed by the library)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step_once()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tsum, ncalls = ctx.timing_totals()
    ncalls = max(ncalls, 1)
    hot, tot, cx = [tsum.hot_ms / ncalls], [tsum.total_ms / ncalls], [tsum.reduce_ms / ncalls]
    cls, rows_k = [tsum.decode_ms / ncalls], [tsum.grid_ms / ncalls]
    st = o["st"].cpu().numpy()
    ql = o["ql"].cpu().numpy().astype(np.int64)
    vl = o["vl"].cpu().numpy().astype(np.int64)
    # input cell bytes + output compacted bytes
    row_q = np.diff(b.row_qual_off.astype(np.int64))
    row_v = np.diff(b.row_val_off.astype(np.int64))
    n_cx = int(out.n_complex)
    alg_all = int(row_q.sum() + row_v.sum() + ql.sum() + vl.sum())
    cells = int(b.kv_qual_len.astype(np.int64).sum() // 2)
    # the roofline is the whole call's: every kernel of tsdbhip_compact_rows
    # (qualifier / value copies, classification, the LDS row kernel for the
    # non-plain rows, complex rows, duplicate decisions) between the call's
    # first and last HIP event (the copies alone overstate it)
    call_ms = float(np.mean(tot))
    hot_ms = float(np.mean(hot))
    nn = lambda v: None if v != v else v  # noqa: E731  (NaN -> null)
    achieved = alg_all / (max(call_ms, 1e-9) * 1e-3) / 1e9
    # (the per-kernel breakdown needs boundary events, which hold each next
    # kernel back ~4.6 us: only under --option timing_detail=on)
    detail = any(o.startswith("timing_detail=") and not o.endswith(("=off", "=0")) for o in args.option)
    if not detail:
        hot, cx, cls, rows_k = [float("nan")], [float("nan")], [float("nan")], [float("nan")]
    kname = "tsdbhip_compact_rows (whole call)"
    call_kernels = "+".join(C5_KERNELS)
    traffic, traffic_src = pmc_traffic("c5", call_kernels, 1)
    res = {
        "metric": "raw cells/sec compacted (CompactionQueue.compact) + % HBM roofline, 1 MI355X",
        "value": cells / (elapsed / args.steps), "unit": "raw cells/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": f"synthetic HBase rows in the reference byte encoding (host-generated in {gen_s:.0f} s, "
                f"HBM-resident before timing)",
        "config": {"workload": CONFIGS["c5"]["desc"], "n_rows": R, "n_kvs": b.n_kvs, "raw_cells": cells,
                   "rows_complex": n_cx, "status_counts": np.bincount(st, minlength=6).tolist()},
        "roofline": {"bound": "hbm", "kernel": kname, "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "traffic_source": traffic_src, "traffic_kernels": call_kernels,
                     "alg_bytes_per_launch": alg_all, "kernel_ms": call_ms,
                     "copy_kernels_ms": nn(hot_ms),
                     "copy_kernels_achieved": nn(alg_all / (max(hot_ms, 1e-9) * 1e-3) / 1e9),
                     "complex_kernel_ms": nn(float(np.mean(cx))), "classify_kernel_ms": nn(float(np.mean(cls))),
                     "rows_kernel_ms": nn(float(np.mean(rows_k)))},
    }
    if args.h2d:
        try:
            res["h2d"] = h2d_leg_c5(ctx, L, b)
        except Exception as e:  # diagnostics only; never costs the line
            res["h2d"] = {"error": repr(e)}
    if not args.no_cpu:
        res["cpu_baseline"] = cpu_baseline_c5(b, args.cpu_seconds)
    emit(res)
    ctx.close()


def h2d_leg_c5(ctx, L, b, steps=3):
    """PCIe-inclusive C5 leg — beside the line, never its value: the same
    1M-row batch with the desc and output arrays in registered pinned host
    memory (as CompactionQueue's JNI bridge would hand them over), so every
    call stages the rows H2D and brings the compacted rows back D2H."""
    R = b.n_rows
    qcap, vcap = b.qual_extent + 64, b.val_extent + R + 64
    outs = {k: np.zeros(n, dt) for k, n, dt in
            [("st", R, np.uint8), ("qo", R, np.uint64), ("ql", R, np.uint32), ("vo", R, np.uint64),
             ("vl", R, np.uint32), ("q", qcap, np.uint8), ("v", vcap, np.uint8), ("w", R, np.uint8),
             ("k", R, np.int32)]}
    ins = [b.row_kv_start, b.row_qual_off, b.row_val_off, b.kv_qual_len, b.kv_val_len, b.qual_bytes, b.val_bytes]
    reg = [a for a in ins + list(outs.values()) if a.nbytes]
    for a in reg:
        ctx.check(L.tsdbhip_host_register(ctx.handle, a.ctypes.data_as(C.c_void_p), a.nbytes))
    try:
        d = _abi.RowsDesc(flags=0, n_rows=R, n_kvs=b.n_kvs, row_kv_start=_abi.ptr(b.row_kv_start, C.c_uint64),
                          row_qual_off=_abi.ptr(b.row_qual_off, C.c_uint64),
                          row_val_off=_abi.ptr(b.row_val_off, C.c_uint64),
                          kv_qual_len=_abi.ptr(b.kv_qual_len, C.c_uint16), kv_val_len=_abi.ptr(b.kv_val_len, C.c_uint16),
                          qual_bytes=_abi.ptr(b.qual_bytes, C.c_uint8), qual_nbytes=len(b.qual_bytes),
                          val_bytes=_abi.ptr(b.val_bytes, C.c_uint8), val_nbytes=len(b.val_bytes))
        o = outs
        out = _abi.RowsOut(qual_capacity=qcap, val_capacity=vcap, row_status=_abi.ptr(o["st"], C.c_uint8),
                           row_qual_off=_abi.ptr(o["qo"], C.c_uint64), row_qual_len=_abi.ptr(o["ql"], C.c_uint32),
                           row_val_off=_abi.ptr(o["vo"], C.c_uint64), row_val_len=_abi.ptr(o["vl"], C.c_uint32),
                           qual_bytes=_abi.ptr(o["q"], C.c_uint8), val_bytes=_abi.ptr(o["v"], C.c_uint8),
                           row_write=_abi.ptr(o["w"], C.c_uint8), row_keep_kv=_abi.ptr(o["k"], C.c_int32))
        ctx.check(L.tsdbhip_compact_rows(ctx.handle, C.byref(d), C.byref(out)))  # warm-up
        t0 = time.perf_counter()
        for _ in range(steps):
            ctx.check(L.tsdbhip_compact_rows(ctx.handle, C.byref(d), C.byref(out)))
        dt = (time.perf_counter() - t0) / steps
    finally:
        for a in reg:
            L.tsdbhip_host_unregister(ctx.handle, a.ctypes.data_as(C.c_void_p))
    h2d = sum(a.nbytes for a in ins)
    d2h = sum(a.nbytes for a in outs.values())
    cells = int(b.kv_qual_len.astype(np.int64).sum() // 2)
    return {"value": cells / dt, "unit": "raw cells/s", "ms_per_step": dt * 1e3, "h2d_bytes_per_step": h2d,
            "d2h_bytes_per_step": d2h, "effective_GBs": (h2d + d2h) / dt / 1e9, "steps": steps,
            "pinned_h2d_GBs": pinned_h2d_rate(h2d),
            "sample": "the whole C5 batch, desc and output arrays in registered pinned host memory"}


def shard_ranges(n_series, world):
    """Contiguous span ranges, one per rank, span (TreeMap) order preserved."""
    return [(n_series * r // world, n_series * (r + 1) // world) for r in range(world)]


def timed_loop(step_once, sync, barrier, steps, warmup, after_step=None, before_timed=None):
    """W untimed steps, then exactly K steps bracketed by barrier + device
    sync on both sides; returns this rank's elapsed seconds. before_timed():
    after the warm-up, ahead of the opening barrier."""
    for _ in range(warmup):
        step_once()
    if before_timed:
        before_timed()
    barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step_once()
        if after_step:
            after_step()
    sync()
    elapsed = time.perf_counter() - t0
    barrier()
    return elapsed


def max_over_ranks(dist, x):
    if dist is None:
        return x
    import torch as _t
    t = _t.tensor([x], dtype=_t.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def h2d_leg(ctx, L, cfg, n_spans, steps=3):
    """PCIe-inclusive rate — reported beside the line, never its `value`: the
    same SpanGroup shape with its row bytes in pinned host memory (registered
    with tsdbhip_host_register, as the JNI bridge registers its
    DirectByteBuffers), so every call stages them H2D before
    the kernels run. A bounded sample of the workload (n_spans series)."""
    d = _abi.SgDesc()
    p = _abi.SynthParams(seed=3, n_spans=n_spans, n_points=cfg["n_points"], t0=synth.T0, step=cfg["step"],
                         kind=cfg["kind"], span0=0)
    ctx.check(L.tsdbhip_synth_generate(ctx.handle, C.byref(p), C.byref(d)))
    S, R = int(d.n_spans), int(d.n_rows)
    arrs = [np.empty(S + 1, np.uint64), np.empty(R, np.uint32), np.empty(R, np.uint32), np.empty(R, np.uint64),
            np.empty(R, np.uint64), np.empty(R, np.uint32), np.empty(int(d.qual_nbytes), np.uint8),
            np.empty(int(d.val_nbytes), np.uint8)]
    ctx.check(L.tsdbhip_desc_download(ctx.handle, C.byref(d), *[a.ctypes.data_as(C.c_void_p) for a in arrs]))
    L.tsdbhip_synth_free(ctx.handle, C.byref(d))
    reg = [a for a in arrs if a.nbytes]
    for a in reg:
        ctx.check(L.tsdbhip_host_register(ctx.handle, a.ctypes.data_as(C.c_void_p), a.nbytes))
    try:
        h = _abi.SgDesc()
        h.n_spans, h.n_rows = S, R
        h.span_row_start = _abi.ptr(arrs[0], C.c_uint64)
        h.row_base = _abi.ptr(arrs[1], C.c_uint32)
        h.row_ncells = _abi.ptr(arrs[2], C.c_uint32)
        h.row_qual_off = _abi.ptr(arrs[3], C.c_uint64)
        h.row_val_off = _abi.ptr(arrs[4], C.c_uint64)
        h.row_val_len = _abi.ptr(arrs[5], C.c_uint32)
        h.qual_bytes, h.qual_nbytes = _abi.ptr(arrs[6], C.c_uint8), arrs[6].nbytes
        h.val_bytes, h.val_nbytes = _abi.ptr(arrs[7], C.c_uint8), arrs[7].nbytes
        h.flags = 0
        h.start_time, h.end_time = 0, (1 << 32) - 1
        h.agg, h.rate, h.ds_interval, h.ds_agg = cfg["agg"], int(cfg["rate"]), cfg["dsi"], cfg["dsa"]
        cap = max(1, cfg["n_points"] * max(cfg["step"], 1))
        ts, isi, bits = np.zeros(cap, np.int64), np.zeros(cap, np.uint8), np.zeros(cap, np.int64)
        out = _abi.SgOut(capacity=cap, ts=_abi.ptr(ts, C.c_int64), is_int=_abi.ptr(isi, C.c_uint8),
                         bits=_abi.ptr(bits, C.c_int64))
        ctx.check(L.tsdbhip_spangroup_run(ctx.handle, C.byref(h), C.byref(out)))  # warm-up
        t0 = time.perf_counter()
        for _ in range(steps):  # each call returns after its D2H of the results
            ctx.check(L.tsdbhip_spangroup_run(ctx.handle, C.byref(h), C.byref(out)))
        dt = (time.perf_counter() - t0) / steps
    finally:
        for a in reg:
            L.tsdbhip_host_unregister(ctx.handle, a.ctypes.data_as(C.c_void_p))
    nbytes = sum(a.nbytes for a in arrs)
    return {"value": int(out.n_input_points) / dt, "unit": "input points/s", "ms_per_step": dt * 1e3,
            "h2d_bytes_per_step": nbytes, "effective_GBs": nbytes / dt / 1e9, "steps": steps,
            "pinned_h2d_GBs": pinned_h2d_rate(nbytes),
            "sample": f"{S} series of the same workload, desc arrays in registered pinned host memory "
                      "(staged H2D inside every call)"}


def pinned_h2d_rate(nbytes, reps=5):
    """This box's plain pinned host -> HBM copy rate for a buffer of `nbytes`
    (the ceiling of any host-resident leg): best of `reps` copies."""
    import torch
    src = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    best = 0.0
    for _ in range(reps):
        t0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        best = max(best, nbytes / (time.perf_counter() - t0) / 1e9)
    del src, dst
    return best


def spawn_ranks(n):
    """`python bench.py --gpus N` without a launcher: run the same command as
    N ranks of torch.distributed.run on this node (127.0.0.1 rendezvous) as
    a child process; its rank 0 prints the line."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3s", choices=sorted(CONFIGS))
    ap.add_argument("--series", type=int, default=0, help="override the number of series")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--exact", action="store_true", help="TSDBHIP_EXACT_ORDER")
    ap.add_argument("--groups", type=int, default=0, help="GROUP BY: split the series into this many SpanGroups "
                    "(tsdbhip_spangroup_run_batch)")
    ap.add_argument("--h2d", action="store_true", help="add the PCIe-inclusive leg (host-resident desc in "
                    "registered pinned memory, 100k-series sample; reported beside the line, never its value)")
    ap.add_argument("--c5-mix", default="c5", choices=["c5", "plain", "nocomplex"],
                    help="C5 row mix (diagnostics; the C5 line is 'c5')")
    ap.add_argument("--rehearse-shards", type=int, default=0,
                    help="diagnostic at N=1: run rank 0's shard of an N-way series split through the sharded "
                         "path on a 1-rank RCCL communicator (per-rank work and exchange code of an N-GPU run; "
                         "the line says so and its value is that one shard's rate)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="a context option (tsdbhip_set_option: decode, aligned_group, lockstep, compact, events, "
                         "timing_detail) for A/B runs; results never depend on it")
    ap.add_argument("--dry-run", action="store_true",
                    help="harness check without a GPU: the multi-rank timing/barrier/report path with a "
                         "no-op step (its value is meaningless and says so)")
    args = ap.parse_args()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        # one process per GPU: start the N ranks under torch.distributed.run
        # (before anything here touches a GPU) and exit with their status
        sys.exit(spawn_ranks(args.gpus))
    if world_env is not None and int(world_env) != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}", file=sys.stderr)
        sys.exit(2)
    global _JSON_OUT
    sys.stdout.flush()
    _JSON_OUT = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    if args.config == "c5":
        return bench_c5(args)

    dist, rank, world, local_rank = dist_setup(args.gpus)
    cfg = CONFIGS[args.config]
    n_series, n_points, step, kind = cfg["n_series"], cfg["n_points"], cfg["step"], cfg["kind"]
    agg, dsi, dsa, rate, desc_txt = cfg["agg"], cfg["dsi"], cfg["dsa"], cfg["rate"], cfg["desc"]
    if args.series:
        n_series = args.series
        cfg = dict(cfg, n_series=n_series)
    if args.groups:
        cfg = dict(cfg, groups=args.groups)
    G = cfg["groups"]
    if G > 1:
        # GROUP BY: groups are independent SpanGroups, so ranks take whole
        # groups (contiguous, group order kept) and exchange nothing
        gb = [n_series * g // G for g in range(G + 1)]
        granks = shard_ranges(G, world)
        shards = [(gb[a], gb[b]) for a, b in granks]
        g_lo, g_hi = granks[rank]
    else:
        shards = shard_ranges(n_series, world)
    rehearse = args.rehearse_shards if (world == 1 and G == 1 and args.rehearse_shards > 1) else 0
    if rehearse:
        shards = shard_ranges(n_series, rehearse)
    lo, hi = shards[rank]

    def barrier():
        if dist is not None:
            dist.barrier()

    if args.dry_run:
        elapsed = max_over_ranks(dist, timed_loop(lambda: time.sleep(0.001), lambda: None, barrier,
                                                   args.steps, args.warmup))
        if rank == 0:
            emit({"metric": METRIC, "value": n_series * n_points / (elapsed / args.steps),
                              "unit": "input points/s", "n_gpus": world, "steps": args.steps,
                              "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                              "dry_run": True, "config": {"workload": desc_txt, "shards": shards}})
        if dist is not None:
            dist.destroy_process_group()
        return

    import torch
    torch.cuda.set_device(local_rank)
    ctx = Context(local_rank)
    set_options(ctx, args.option)
    L = lib()
    if world > 1:
        uid = [Context.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        ctx.comm_init(world, rank, uid[0])
    elif rehearse:
        ctx.comm_init(1, 0, Context.unique_id())

    d = _abi.SgDesc()
    keep = []
    if cfg["gen"] == "device":  # the reference's byte format generated straight into HBM
        p = _abi.SynthParams(seed=3, n_spans=hi - lo, n_points=n_points, t0=synth.T0, step=step,
                             kind=kind, span0=lo)
        ctx.check(L.tsdbhip_synth_generate(ctx.handle, C.byref(p), C.byref(d)))
        local_bytes = ref_row_bytes(hi - lo, n_points, step, kind)
    else:  # host-generated (jittered C4 shapes), uploaded to HBM before timing
        ss = host_spanset(cfg, lo, hi)
        dev = torch.device("cuda", local_rank)

        def up(arr, ctype):
            t = torch.from_numpy(np.ascontiguousarray(arr).view(np.uint8)).to(dev)
            keep.append(t)
            return C.cast(C.c_void_p(t.data_ptr()), C.POINTER(ctype))

        ss.fill_desc(d)
        d.flags = _abi.DESC_DEVICE
        d.span_row_start = up(ss.span_row_start, C.c_uint64)
        d.row_base = up(ss.row_base, C.c_uint32)
        d.row_ncells = up(ss.row_ncells, C.c_uint32)
        d.row_qual_off = up(ss.row_qual_off, C.c_uint64)
        d.row_val_off = up(ss.row_val_off, C.c_uint64)
        d.row_val_len = up(ss.row_val_len, C.c_uint32)
        d.qual_bytes = up(ss.qual_bytes, C.c_uint8)
        d.val_bytes = up(ss.val_bytes, C.c_uint8)
        local_bytes = spanset_row_bytes(ss)
        n_points = int(cfg["n_points"] * 1.5 * n_series)  # bound on the union grid
    d.start_time = 0
    d.end_time = (1 << 32) - 1
    d.agg, d.rate, d.ds_interval, d.ds_agg = agg, int(rate), dsi, dsa
    if (world > 1 or rehearse) and G == 1:
        d.flags |= _abi.SHARDED
        d.span0 = lo
    if args.exact:
        d.flags |= _abi.EXACT_ORDER
    if cfg["gen"] == "device":
        cap = max(1, n_points if dsi == 0 else (n_points * step) // dsi + 2)
    else:  # union of all timestamps (bounded by all ranks' input points)
        cap = max(1, n_points + 16)
    ts = np.zeros(cap, np.int64)
    isi = np.zeros(cap, np.uint8)
    bits = np.zeros(cap, np.int64)
    out = _abi.SgOut(capacity=cap, ts=_abi.ptr(ts, C.c_int64), is_int=_abi.ptr(isi, C.c_uint8),
                     bits=_abi.ptr(bits, C.c_int64))

    def pin(*arrs):
        # result buffers page-locked, as the JNI bridge registers its
        # DirectByteBuffers (tsdbhip_host_register): the D2H
        # of a large result is then one DMA
        for a in arrs:
            if a.nbytes:
                ctx.check(L.tsdbhip_host_register(ctx.handle, a.ctypes.data_as(C.c_void_p), a.nbytes))

    pin(ts, isi, bits)

    def step_once():
        ctx.check(L.tsdbhip_spangroup_run(ctx.handle, C.byref(d), C.byref(out)))

    if G > 1:
        Gl = g_hi - g_lo
        gss = np.array([gb[g] - lo for g in range(g_lo, g_hi + 1)], np.uint32)
        gcap = cap
        g_ts = np.zeros(Gl * gcap, np.int64)
        g_isi = np.zeros(Gl * gcap, np.uint8)
        g_bits = np.zeros(Gl * gcap, np.int64)
        pin(g_ts, g_isi, g_bits)
        outs = (_abi.SgOut * Gl)()
        for g in range(Gl):
            outs[g].capacity = gcap
            outs[g].ts = _abi.ptr(g_ts[g * gcap:], C.c_int64)
            outs[g].is_int = _abi.ptr(g_isi[g * gcap:], C.c_uint8)
            outs[g].bits = _abi.ptr(g_bits[g * gcap:], C.c_int64)

        def step_once():
            ctx.check(L.tsdbhip_spangroup_run_batch(ctx.handle, C.byref(d), Gl, _abi.ptr(gss, C.c_uint32), outs))

    # per-call HIP-event timings of the timed steps, summed by the library
    # (tsdbhip_timing_totals: no readout call inside the timed loop)
    elapsed = max_over_ranks(dist, timed_loop(step_once, torch.cuda.synchronize, barrier, args.steps,
                                              args.warmup, before_timed=lambda: ctx.timing_totals(reset=True)))
    tsum, ncalls = ctx.timing_totals()
    ncalls = max(ncalls, 1)
    hot_ms, total_ms, red_ms = [tsum.hot_ms / ncalls], [tsum.total_ms / ncalls], [tsum.reduce_ms / ncalls]
    emitted = [int(tsum.n_emitted) // ncalls, int(tsum.n_grid) // ncalls]
    hot_kernel = tsum.hot_kernel
    # achievable bandwidth on this box, same buffers (tsdbhip_bw_probe): a
    # streaming read with the downsampler's geometry and a D2D copy
    probe = {}
    width = 4 if kind == _abi.SYN_FLOAT32 else 8
    for mode, name in (((0, "read_stream"), (1, "d2d_copy")) if cfg["gen"] == "device" else ()):
        ms, nb = C.c_float(), C.c_uint64()
        best = None
        for _ in range(3):
            ctx.check(L.tsdbhip_bw_probe(ctx.handle, C.byref(d), mode, width, C.byref(ms), C.byref(nb)))
            gbs = nb.value / (ms.value * 1e-3) / 1e9
            best = gbs if best is None else max(best, gbs)
        probe[name] = best
    n_input = int(out.n_input_points)  # global (allreduced when sharded)
    if G > 1:  # groups sharded: each rank's own points, summed over ranks
        n_input = sum(int(outs[g].n_input_points) for g in range(Gl))
        if dist is not None:
            import torch as _t
            t = _t.tensor([n_input], dtype=_t.float64)
            dist.all_reduce(t)
            n_input = int(t.item())
    ms_step = elapsed / args.steps * 1e3
    value = n_input / (elapsed / args.steps)
    late_total = int(tsum.late_stamp)
    if dist is not None:
        import torch as _t
        t = _t.tensor([late_total], dtype=_t.int64)
        dist.all_reduce(t)
        late_total = int(t.item())

    # roofline of the dominant kernel: SURVEY.md §8(d) algorithmic bytes (the
    # row bytes it streams) over its own duration (HIP events on its stream)
    hot = float(np.mean(hot_ms))
    kname = _abi.HOT_NAMES.get(hot_kernel, "none")
    hot_bytes = local_bytes
    if kname == "k_reduce":  # direct path: the reducer streams the value bytes only
        if cfg["gen"] == "device":
            hot_bytes = (hi - lo) * cfg["n_points"] * width
        else:
            nc = ss.row_ncells.astype(np.int64)
            hot_bytes = int((ss.row_val_len.astype(np.int64) - (nc > 1)).sum())
    reduce_ms = float(np.mean(red_ms))
    valu_bound = False
    if G == 1 and kname != "k_reduce" and reduce_ms > 2 * hot:
        # the cross-span reducer dominates (C4: VALU-bound lerps): roofline on
        # it, with its algorithmic bytes = the E points it reads (u32 ts, i64
        # bits, u8 flag) + the output it writes (T x 17 B)
        kname, hot = "k_reduce", reduce_ms
        hot_bytes = emitted[0] * 13 + emitted[1] * 17
        valu_bound = True
    achieved = hot_bytes / (max(hot, 1e-9) * 1e-3) / 1e9
    # (the committed PMC passes are whole-config, one GPU: a rehearsed shard
    # has no traffic figure of its own)
    traffic, traffic_src = pmc_traffic(args.config, kname, max(world, rehearse))
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": value,
            "unit": "input points/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int64" if (kind == _abi.SYN_INT64_COUNTER and not rate) or cfg["gen"] == "jitter_int"
                     else "f64",
            "data": "synthetic (device-generated KeyValue bytes in the reference encoding)",
            "config": {
                "workload": desc_txt,
                "n_series": n_series,
                "points_per_series": cfg["n_points"],
                "rate": bool(rate),
                "aggregator": ["sum", "min", "max", "avg", "dev"][agg],
                "downsample": f"{dsi}s-{['sum', 'min', 'max', 'avg', 'dev'][dsa]}" if dsi else "none",
                "parallelism": (f"groups-sharded x{world} (independent SpanGroups, no exchange)" if G > 1
                                else f"series-sharded x{world} (RCCL exchange of per-t partials)") if world > 1
                               else "single GPU",
                "groups": G,
                "shards": shards,
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kname,
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "alg_bytes_per_launch": hot_bytes,
                "kernel_ms": hot,
                "step_device_ms": float(np.mean(total_ms)),
                "path_alg_bytes": local_bytes,
                "path_GBs": local_bytes / (max(float(np.mean(total_ms)), 1e-9) * 1e-3) / 1e9,
                "achievable_GBs": {k: round(v, 1) for k, v in probe.items()},
                "frac_of_read_stream": achieved / probe["read_stream"] if probe else None,
            },
        }
        if valu_bound:
            # C4: lerps on E spans make the reducer VALU-bound, so its roofline
            # is the VALU issue rate (SQ_INSTS_VALU per launch from the
            # committed PMC pass of this config over the live kernel time);
            # the HBM figures stay beside it
            vi, vsrc = pmc_valu(args.config, "k_reduce")
            rl = res["roofline"]
            rl["hbm"] = {k: rl.pop(k) for k in ("achieved", "peak", "unit", "frac")}
            rl["bound"] = "valu"
            rl["unit"] = "wave-instr/s"
            rl["peak"] = VALU_PEAK_WIPS
            rl["valu_insts_per_launch"] = vi
            rl["valu_source"] = vsrc
            rl["achieved"] = vi / (hot * 1e-3) if vi and hot > 0 else None
            rl["frac"] = rl["achieved"] / VALU_PEAK_WIPS if vi else None
        # which variants ran (tsdbhip_timing.paths): the aligned-group reduction
        # (k_ds_reg's block partials instead of E + k_reduce) or its rerun
        res["paths"] = {"aligned_group": bool(tsum.paths & _abi.PATH_ALIGNED_GROUP),
                        "aligned_rerun": bool(tsum.paths & _abi.PATH_ALIGNED_RERUN)}
        if world > 1 or rehearse:  # collective launches per call on this rank (RCCL groups)
            res["collectives_per_call"] = tsum.n_collectives / ncalls
        # timed calls whose call-end stamp (the host's proof that the snapshot
        # and results are this call's) arrived only after the stream sync,
        # summed over the ranks
        res["late_stamp"] = {"calls": late_total, "of": ncalls * world}
        if rehearse:
            res["rehearsal"] = {"shards": rehearse, "note": f"shard 0 of {rehearse} on a 1-rank RCCL "
                                "communicator; value = this shard's points/s, not a node figure"}
            res["config"]["parallelism"] = f"rehearsal: 1 of {rehearse} series shards"
        if args.h2d and world == 1 and cfg["gen"] == "device" and G == 1:
            try:
                res["h2d"] = h2d_leg(ctx, L, cfg, min(n_series, 100_000))
            except Exception as e:  # diagnostics only; never costs the line
                res["h2d"] = {"error": repr(e)}
        if not args.no_cpu and world == 1 and not rehearse:
            res["cpu_baseline"] = cpu_baseline(args.config, args.cpu_seconds)
        emit(res)
    if cfg["gen"] == "device":
        L.tsdbhip_synth_free(ctx.handle, C.byref(d))
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
