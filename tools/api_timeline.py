"""One step's host-API + kernel timeline from a rocprofv3 run with
--kernel-trace --hip-runtime-trace (csv):
python tools/api_timeline.py gpurun_out/tapi/c1/run [anchor-api] [nth-from-last]
A step starts at an anchor kernel launch (default: the k_assemble_fast
launch) and runs to the next one."""
import csv
import sys

pre = sys.argv[1]
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_assemble_fast"
nth = int(sys.argv[3]) if len(sys.argv) > 3 else 2
api = list(csv.DictReader(open(pre + "_hip_api_trace.csv")))
ker = list(csv.DictReader(open(pre + "_kernel_trace.csv")))
kc = {k["Correlation_Id"]: k for k in ker}
# anchor kernels by start time
ak = sorted((int(k["Start_Timestamp"]), k) for k in ker if anchor in k["Kernel_Name"])
s0, s1 = ak[-nth - 1][0], ak[-nth][0]
a0 = int([a for a in api if a["Correlation_Id"] == ak[-nth - 1][1]["Correlation_Id"]][0]["Start_Timestamp"])
a1 = int([a for a in api if a["Correlation_Id"] == ak[-nth][1]["Correlation_Id"]][0]["Start_Timestamp"])
ev = []
for a in api:
    s, e = int(a["Start_Timestamp"]), int(a["End_Timestamp"])
    if a0 <= s < a1:
        ev.append((s, e, "API", a["Function"], a["Correlation_Id"]))
for k in ker:
    s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
    if s0 <= s < s1:
        ev.append((s, e, "GPU", k["Kernel_Name"].split("(")[0][:60], k["Correlation_Id"]))
t0 = min(a0, s0)
busy = 0
for s, e, kind, name, cid in sorted(ev):
    if kind == "GPU":
        busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  {kind} {name}")
print(f"host step {(a1 - a0) / 1e3:.1f} us, gpu step {(s1 - s0) / 1e3:.1f} us, kernels busy {busy / 1e3:.1f} us")
