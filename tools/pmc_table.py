#!/usr/bin/env python3
"""Summarise tools/gpu/pmc_passes.sh output (gpurun_out/pmc/<config>/): per
kernel, the average duration (kernel trace), every counter of the passes per
launch, the HBM bytes per launch corrected as MI355X_MICROARCH.md §HBM
prescribes (2 x FETCH_SIZE + WRITE_SIZE, KiB), and the derived limiter
figures: VALU issue against the VALU peak, wait / VALU-active / LDS-active
shares of the wave-cycles, LDS bank conflicts per LDS instruction, L2 hit
rate. The JSON has bench.py's profiles/pmc_<config>.json keys (avg_ms,
calls, fetch_kib_raw, write_kib, hbm_bytes_per_launch, valu_insts_per_launch)
plus "counters" and "derived".

usage: pmc_table.py gpurun_out/pmc/<config> [tag] > profiles/pmc_<config>.json
       pmc_table.py --text gpurun_out/pmc/<config>   (a table, largest first)
"""
import collections
import csv
import glob
import json
import os
import sys

VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2  # wave-instructions/s (as bench.py / diag_summary.py)


def short(n):
    return n.split("(")[0].replace("void ", "").replace("tsdb::", "").strip()


def counters(root):
    """{kernel: {counter: average over dispatches of the value summed over its rows}}"""
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
    for f in glob.glob(os.path.join(root, "*", "**", "run_counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            acc[short(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def summary(root, tag):
    out = {"tag": tag, "kernels": {}}
    stats = glob.glob(os.path.join(root, "trace", "**", "run_kernel_stats.csv"), recursive=True)
    if stats:
        for r in csv.DictReader(open(stats[0])):
            e = out["kernels"].setdefault(short(r["Name"]), {})
            e["avg_ms"] = float(r["AverageNs"]) / 1e6
            e["calls"] = int(r["Calls"])
    for k, c in counters(root).items():
        e = out["kernels"].setdefault(k, {})
        e["counters"] = c
        if "SQ_INSTS_VALU" in c:
            e["valu_insts_per_launch"] = c["SQ_INSTS_VALU"]
        f, w = c.get("FETCH_SIZE"), c.get("WRITE_SIZE")
        e["fetch_kib_raw"] = f
        e["write_kib"] = w
        if f is not None and w is not None:
            e["hbm_bytes_per_launch"] = 2.0 * f * 1024.0 + w * 1024.0
        d = {}
        t = e.get("avg_ms")
        if t and "SQ_INSTS_VALU" in c:
            d["valu_issue_frac"] = c["SQ_INSTS_VALU"] / (VALU_PEAK_WIPS * t / 1e3)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc:
            for name, key in (("wait_inst_any", "SQ_WAIT_INST_ANY"), ("wait_any", "SQ_WAIT_ANY"),
                              ("active_valu", "SQ_ACTIVE_INST_VALU"), ("active_any", "SQ_ACTIVE_INST_ANY"),
                              ("active_lds", "SQ_ACTIVE_INST_LDS"), ("wait_lds", "SQ_WAIT_INST_LDS")):
                if key in c:
                    d[name + "_of_wave_cycles"] = c[key] / wc
        if c.get("SQ_INSTS_LDS"):
            d["lds_bank_conflict_cycles_per_lds_inst"] = c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_INSTS_LDS"]
        h, m = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            d["l2_hit_rate"] = h / (h + m)
        if c.get("SQ_WAVES") and wc and t:
            d["avg_resident_waves"] = 4 * wc / (t * 1e-3 * 2.4e9)  # (SQ_WAVE_CYCLES counts quad-cycles on gfx9: x4)
        e["derived"] = d
    return out


def text(s):
    ks = sorted(s["kernels"].items(), key=lambda kv: -(kv[1].get("avg_ms") or 0) * (kv[1].get("calls") or 0))
    for k, e in ks[:12]:
        d = e.get("derived", {})
        hbm = e.get("hbm_bytes_per_launch")
        ms = e.get("avg_ms") or 0
        line = f"{ms:8.3f} ms {k[:40]:40s}"
        if hbm and ms:
            line += f" HBM {hbm / 1e9:6.3f} GB ({hbm / (ms * 1e-3) / 1e12:5.2f} TB/s)"
        for key, lab in (("valu_issue_frac", "valu"), ("wait_inst_any_of_wave_cycles", "wait"),
                         ("active_lds_of_wave_cycles", "lds"), ("lds_bank_conflict_cycles_per_lds_inst", "bankc"),
                         ("l2_hit_rate", "L2hit")):
            if key in d:
                line += f" {lab} {d[key]:.2f}"
        print(line)


def main():
    if sys.argv[1] == "--text":
        root = sys.argv[2]
        text(summary(root, os.path.basename(root.rstrip("/"))))
        return
    root = sys.argv[1]
    tag = sys.argv[2] if len(sys.argv) > 2 else os.path.basename(root.rstrip("/"))
    json.dump(summary(root, tag), sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main()
