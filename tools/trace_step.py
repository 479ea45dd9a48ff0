"""Print one step's kernel timeline from a rocprofv3 kernel-trace CSV.

usage: python tools/trace_step.py run_kernel_trace.csv ANCHOR_SUBSTRING [pre]
The step shown starts `pre` dispatches before the second-to-last launch whose
name contains ANCHOR and ends just before the same point of the next step.
"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2]
pre = int(sys.argv[3]) if len(sys.argv) > 3 else 12
idx = [i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]]
seg = rows[idx[-3] - pre: idx[-2] - pre + 1]
t0 = int(seg[0]["Start_Timestamp"])
prev = None
for r in seg:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print("%9.1f us dur %7.1f gap %6.1f %s" % ((s - t0) / 1e3, (e - s) / 1e3, gap, r["Kernel_Name"][:80]))
    prev = e
