#!/bin/bash
# instruction mix + HBM bytes per kernel for one bench config: pmc_cfg.sh <config> <out>
set -e
CFG=$1; OUT=gpurun_out/$2
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM"
P2="SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o run -- python3 bench.py --config $CFG --no-cpu --steps 1 --warmup 1 > $OUT/p$i.log 2>&1
done
python3 - $OUT <<'PY'
import csv, collections, glob, sys
out = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(out + "/p*/run_counter_collection.csv")):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        per[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (k, c, d), v in per.items():
        acc[k][c].append(v)
for k, cs in acc.items():
    if "k_probe" in k or "synth" in k: continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):.4g}")
PY
