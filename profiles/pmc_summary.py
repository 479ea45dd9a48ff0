#!/usr/bin/env python3
"""Summarise a profiles/profile.sh run: per kernel, the average duration
from the kernel trace and the HBM traffic per launch from the PMC passes,
corrected as MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE reports half
the bytes of wide coalesced streaming reads on gfx950 -> x2; WRITE_SIZE is
exact for 16-B/lane stores; both are in KiB).

usage: pmc_summary.py <prof dir> [config tag] > summary.json
"""
import collections
import csv
import json
import os
import sys


def short(name):
    n = name.split("(")[0]
    for pre in ("void ", "tsdb::"):
        n = n.replace(pre, "")
    return n.strip()


def per_dispatch(path, counter):
    """{kernel: average over dispatches of the counter summed over its rows}"""
    if not os.path.exists(path):
        return {}
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[short(r["Kernel_Name"])][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in acc.items()}


def main():
    d = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(d.rstrip("/"))
    out = {"tag": tag, "kernels": {}}
    stats = os.path.join(d, "trace", "run_kernel_stats.csv")
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            out["kernels"].setdefault(short(r["Name"]), {})["avg_ms"] = float(r["AverageNs"]) / 1e6
            out["kernels"][short(r["Name"])]["calls"] = int(r["Calls"])
    valu = per_dispatch(os.path.join(d, "pmc_sq", "run_counter_collection.csv"), "SQ_INSTS_VALU")
    for k, v in valu.items():  # VALU wave-instructions per launch (VALU-bound kernels' roofline)
        out["kernels"].setdefault(k, {})["valu_insts_per_launch"] = v
    fetch = per_dispatch(os.path.join(d, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(d, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    for k in set(fetch) | set(write):
        e = out["kernels"].setdefault(k, {})
        f = fetch.get(k)
        w = write.get(k)
        e["fetch_kib_raw"] = f
        e["write_kib"] = w
        if f is not None and w is not None:
            e["hbm_bytes_per_launch"] = 2.0 * f * 1024.0 + w * 1024.0
    json.dump(out, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
