#!/bin/bash
# instruction mix of the downsampling kernel on C3* (GPU box)
set -e
mkdir -p gpurun_out/exp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d gpurun_out/exp/pmc -o run -- python3 bench.py --config c3s --no-cpu --steps 1 --warmup 1 > gpurun_out/exp/pmc.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/exp/pmc2 -o run -- python3 bench.py --config c3s --no-cpu --steps 1 --warmup 1 > gpurun_out/exp/pmc2.log 2>&1
python3 - <<'PY'
import csv, collections
for f in ["gpurun_out/exp/pmc/run_counter_collection.csv", "gpurun_out/exp/pmc2/run_counter_collection.csv"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_ds_spans" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in acc.items(): print(c, sum(d.values()) / len(d))
PY
