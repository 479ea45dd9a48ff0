#!/bin/bash
# instruction mix / waits of the C5 plain-row kernels (GPU box)
set -e
O=gpurun_out/pmc_c5v
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --output-format csv -d $O/p1 -o run -- python3 bench.py --config c5 --no-cpu --steps 1 --warmup 1 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum --output-format csv -d $O/p2 -o run -- python3 bench.py --config c5 --no-cpu --steps 1 --warmup 1 > $O/p2.log 2>&1
python3 - <<'PY'
import csv, collections
for f in ["gpurun_out/pmc_c5v/p1/run_counter_collection.csv", "gpurun_out/pmc_c5v/p2/run_counter_collection.csv"]:
    for kn in ("k_compact_vals", "k_compact_classify", "k_compact_rows"):
        acc = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(f)):
            if kn not in r["Kernel_Name"]: continue
            acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
        print(kn, {c: round(sum(d.values()) / len(d)) for c, d in acc.items()})
PY
