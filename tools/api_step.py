"""One step of a rocprofv3 --hip-trace --kernel-trace run: host HIP API calls
and kernels on one time axis (us from the step's first kernel launch call).
python tools/api_step.py <dir with *_hip_api_trace.csv and *_kernel_trace.csv> [first kernel]"""
import csv
import glob
import sys

d = sys.argv[1]
first = sys.argv[2] if len(sys.argv) > 2 else "k_assemble_tiles"
api = sorted(csv.DictReader(open(glob.glob(f"{d}/**/*hip_api_trace.csv", recursive=True)[0])),
             key=lambda r: int(r["Start_Timestamp"]))
ker = sorted(csv.DictReader(open(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0])),
             key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(ker) if first in r["Kernel_Name"]]
a, b = idx[-3], idx[-2]
k0, k1 = int(ker[a]["Start_Timestamp"]), int(ker[b]["Start_Timestamp"])
# the launch call of kernel a: the last API call starting before it
calls = [r for r in api if int(r["Start_Timestamp"]) <= k1]
t0 = max(int(r["Start_Timestamp"]) for r in calls if int(r["Start_Timestamp"]) <= k0 and "Launch" in r["Function"])
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r["Function"]) for r in api
      if t0 - 60000 <= int(r["Start_Timestamp"]) < k1]
ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "gpu", r["Kernel_Name"].split("(")[0][:60]) for r in ker[a:b + 1]]
for s, e, kind, name in sorted(ev):
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {kind}  {name}")
