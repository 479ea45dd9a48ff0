#!/bin/bash
# C4 / C4-int after the reducer's cached long lerp: kernel trace + PMC passes
# (profiles/profile.sh), summaries for the bench's VALU roofline (GPU box)
set -e
bash profiles/profile.sh c4 --config c4 --steps 2 --warmup 1
bash profiles/profile.sh c4i --config c4i --steps 2 --warmup 1
python3 - <<'PY'
import json
for t in ("c4", "c4i"):
    d = json.load(open(f"gpurun_out/prof_{t}/summary.json"))
    for k in ("k_reduce", "k_assemble", "k_decode_nods"):
        for n, e in d["kernels"].items():
            if n.split("<")[0] == k:
                print(t, n, round(e.get("avg_ms") or 0, 3), e.get("valu_insts_per_launch"))
PY
