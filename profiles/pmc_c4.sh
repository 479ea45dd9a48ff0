#!/bin/bash
# C4 / C4-int k_reduce instruction mix (GPU box): separate PMC passes
set -e
O=gpurun_out/pmc_c4
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in c4 c4i; do
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/sq_$c -o run -- python3 bench.py --config $c --no-cpu --steps 1 --warmup 1 > $O/sq_$c.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA --output-format csv -d $O/sq2_$c -o run -- python3 bench.py --config $c --no-cpu --steps 1 --warmup 1 > $O/sq2_$c.log 2>&1
done
python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob("gpurun_out/pmc_c4/sq*/run_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_reduce" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(f.split('/')[2], {c: '%.3e' % (sum(d.values()) / len(d)) for c, d in acc.items()})
PY
