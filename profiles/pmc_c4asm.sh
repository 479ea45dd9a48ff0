#!/bin/bash
# instruction mix / waits of k_assemble on C4 (GPU box)
set -e
O=gpurun_out/pmc_c4asm
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d $O/p1 -o run -- python3 bench.py --config c4 --no-cpu --steps 1 --warmup 1 > $O/p1.log 2>&1
python3 - <<'PY'
import csv, collections
for kn in ("k_assemble(", "k_decode_nods", "k_grid_mark"):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open("gpurun_out/pmc_c4asm/p1/run_counter_collection.csv")):
        if kn not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(kn, {c: round(sum(d.values()) / len(d)) for c, d in acc.items()})
PY
