"""BASELINE.md results table from a directory of bench.py JSON lines:
python tools/results_table.py profiles/r02_s2/cfgs"""
import json
import os
import sys

ORDER = [("c1", "C1"), ("c2", "C2"), ("c3", "C3 sum (no rate)"), ("c3r_sum", "C3 rate sum"),
         ("c3r_max", "C3 rate max"), ("c3r_dev", "C3 rate dev"), ("c3s", "C3* (headline)"),
         ("c3s_gb100", "C3* GROUP BY 100"), ("c3s_gb10k", "C3* GROUP BY 10k"), ("c3_gb100", "C3 GROUP BY 100"),
         ("c4", "C4"), ("c4i", "C4-int"), ("c5", "C5"), ("c3_dev", "C3 shape, 1M series, integer dev"),
         ("c3_dev_100k", "C3 shape, 100k series, integer dev")]
PAR = "bit-exact ints; doubles 1e-9 / bit-exact with EXACT_ORDER"
d = sys.argv[1]
print("| config | GPUs | value | ms/step | achieved (dominant kernel) | % of 8 TB/s | CPU value | CPU threads | parity |")
print("|---|---|---|---|---|---|---|---|---|")
for key, name in ORDER:
    f = os.path.join(d, key + ".json")
    if not os.path.exists(f):
        continue
    x = json.loads(open(f).read().strip().splitlines()[-1])
    r, c = x["roofline"], x.get("cpu_baseline") or {}
    unit = "cells/s" if key == "c5" else "pts/s"
    if r.get("bound") == "valu" and r.get("valu_insts_per_launch"):
        ach = (f"{r['kernel']} {r['kernel_ms']:.1f} ms, VALU-bound: {r['valu_insts_per_launch']:.3g} VALU "
               f"wave-instr/launch = {r['achieved']:.2g}/s")
        pct = f"{100 * r['frac']:.0f} % of VALU issue"
    elif r.get("bound") == "valu":
        ach, pct = f"{r['kernel']} {r['kernel_ms']:.1f} ms, VALU-bound", "-"
    elif key != "c5" and r.get("kernel_ms") and r["kernel_ms"] < 0.25 * x["ms_per_step"]:
        # (the dominant kernel is a small share of the step: a roofline of it
        # would describe a fraction of the time)
        ach = (f"launch / latency-bound: {r['kernel']} {r['kernel_ms']:.3f} ms of the "
               f"{x['ms_per_step']:.3f} ms step")
        pct = "-"
    else:
        hbm = r.get("hbm", r)
        ach = f"{hbm['achieved']:.0f} GB/s ({r['kernel']} {r['kernel_ms']:.3f} ms)"
        pct = f"{100 * hbm['achieved'] / 8000:.1f} %"
    par = "bit-exact (full 1M-row batch)" if key == "c5" else PAR
    print(f"| {name} | {x['n_gpus']} | {x['value']:.3g} {unit} | {x['ms_per_step']:.3f} | {ach} | {pct} | "
          f"{c.get('value', float('nan')):.3g} | {c.get('cores', '-')} ({c.get('kind', '-')}) | {par} |")
