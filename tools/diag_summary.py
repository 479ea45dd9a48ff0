#!/usr/bin/env python3
"""Tabulates tools/gpu/diag.sh output: per config and kernel, the average
duration (kernel stats) and, per launch, the SQ counters of the PMC pass
(VALU issue as a fraction of the VALU issue peak over the kernel's time)."""
import collections
import csv
import glob
import os
import sys

VALU_PEAK_WIPS = 256 * 4 * 2.4e9 / 2  # wave-instructions/s (bench.py)


def short(n):
    return n.split("(")[0].replace("void ", "").replace("tsdb::", "").strip()


def main(root):
    for d in sorted(glob.glob(os.path.join(root, "*"))):
        stats = glob.glob(os.path.join(d, "trace", "**", "run_kernel_stats.csv"), recursive=True)
        pmc = glob.glob(os.path.join(d, "pmc_sq", "**", "run_counter_collection.csv"), recursive=True)
        if not stats:
            continue
        print(f"== {os.path.basename(d)}")
        ms = {}
        for r in csv.DictReader(open(stats[0])):
            ms[short(r["Name"])] = (float(r["AverageNs"]) / 1e6, int(r["Calls"]))
        ctr = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
        if pmc:
            for r in csv.DictReader(open(pmc[0])):
                ctr[short(r["Kernel_Name"])][r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        for k, (t, n) in sorted(ms.items(), key=lambda x: -x[1][0] * x[1][1]):
            line = f"  {t:8.3f} ms x{n:<4d} {k[:70]}"
            c = ctr.get(k)
            if c:
                avg = {name: sum(v.values()) / len(v) for name, v in c.items()}
                valu = avg.get("SQ_INSTS_VALU", 0)
                line += (f" | VALU {valu:.3g} ({valu / (VALU_PEAK_WIPS * t / 1e3):.0%} issue)"
                         f" VMEM {avg.get('SQ_INSTS_VMEM', 0):.3g} SALU {avg.get('SQ_INSTS_SALU', 0):.3g}"
                         f" waves {avg.get('SQ_WAVES', 0):.3g}")
                wc = avg.get("SQ_WAVE_CYCLES", 0)
                if wc:
                    line += (f" wait {avg.get('SQ_WAIT_INST_ANY', 0) / wc:.0%}"
                             f" valu-active {avg.get('SQ_ACTIVE_INST_VALU', 0) / wc:.0%} of wave-cycles")
            print(line)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/diag")
