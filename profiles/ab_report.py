import json, os, sys
d = sys.argv[1]
for f in sorted(os.listdir(d)):
    if f.endswith(".log") and not f.startswith("pytest"):
        x = json.loads(open(os.path.join(d, f)).read().strip().splitlines()[-1])
        print(f, "kernel_ms", round(x["roofline"]["kernel_ms"], 3), "ms_per_step", round(x["ms_per_step"], 3))
