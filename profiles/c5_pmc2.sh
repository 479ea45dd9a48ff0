#!/bin/bash
# C5 compaction: kernel trace + instruction-mix counters for the c5 and plain mixes (GPU box)
set -e
O=gpurun_out/c5b
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for mix in c5 plain; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$mix -o run -- python3 bench.py --config c5 --c5-mix $mix --no-cpu --steps 3 --warmup 1 > $O/tr_$mix.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d $O/pmc_sq_$mix -o run -- python3 bench.py --config c5 --c5-mix $mix --no-cpu --steps 2 --warmup 1 > $O/pmc_sq_$mix.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_sq2_$mix -o run -- python3 bench.py --config c5 --c5-mix $mix --no-cpu --steps 2 --warmup 1 > $O/pmc_sq2_$mix.log 2>&1
done
python3 - <<'PY'
import csv, collections, glob
for f in sorted(glob.glob("gpurun_out/c5b/pmc_*/run_counter_collection.csv")):
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "compact_tiles" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    print(f.split('/')[2], {c: '%.3e' % (sum(d.values()) / len(d)) for c, d in acc.items()})
for f in sorted(glob.glob("gpurun_out/c5b/tr_*/run_kernel_stats.csv")):
    for r in list(csv.DictReader(open(f)))[:4]:
        print(f.split('/')[2], r["Name"][:40], r["Calls"], r["AverageNs"])
PY
