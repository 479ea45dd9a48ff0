#!/bin/bash
# instruction-mix counters for the compaction kernels (GPU box)
set -e
mkdir -p gpurun_out/c5
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d gpurun_out/c5/pmc_sq -o run -- python3 bench.py --config c5 --no-cpu --steps 2 --warmup 1 > gpurun_out/c5/pmc_sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/c5/pmc_sq2 -o run -- python3 bench.py --config c5 --no-cpu --steps 2 --warmup 1 > gpurun_out/c5/pmc_sq2.log 2>&1
python3 - <<'PY'
import csv, collections
for f in ["gpurun_out/c5/pmc_sq/run_counter_collection.csv", "gpurun_out/c5/pmc_sq2/run_counter_collection.csv"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        if "compact_tiles" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in acc.items(): print(c, sum(d.values()) / len(d))
PY
