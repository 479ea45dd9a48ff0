#!/bin/bash
# instruction mix of k_ds_spans<FLT> on C2, and the 8-way shard rehearsal (GPU box)
set -e
O=gpurun_out/pmc_c2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d $O/p1 -o run -- python3 bench.py --config c2 --no-cpu --steps 1 --warmup 1 > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE --output-format csv -d $O/p2 -o run -- python3 bench.py --config c2 --no-cpu --steps 1 --warmup 1 > $O/p2.log 2>&1
python3 - <<'PY'
import csv, collections
for f in ["gpurun_out/pmc_c2/p1/run_counter_collection.csv", "gpurun_out/pmc_c2/p2/run_counter_collection.csv"]:
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "k_ds_spans<3, true>" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    for c, d in acc.items(): print(c, sum(d.values()) / len(d))
PY
for n in 8; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 --rehearse-shards $n > $O/rehearse_$n.json 2> $O/rehearse_$n.err
  cut -c1-400 $O/rehearse_$n.json
done
