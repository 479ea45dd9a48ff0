"""Per-step kernel timeline of a rocprofv3 kernel trace (gaps, durations):
python tools/step_trace.py gpurun_out/prof_c2/run_kernel_trace.csv [first-kernel-of-step]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
first = sys.argv[2] if len(sys.argv) > 2 else "k_assemble_fast"
idx = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
t0 = int(rows[a]["Start_Timestamp"])
prev, busy = t0, 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.1f} gap {(s - prev) / 1e3:7.1f} dur {(e - s) / 1e3:8.1f}  {r['Kernel_Name'].split('(')[0][:70]}")
    busy += e - s
    prev = e
print(f"step {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us, {b - a} kernels")
