#!/bin/bash
# kernel trace summary of one bench config: trace_cfg.sh <config>
set -e
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/tr/$1 -o run -- python3 bench.py --no-cpu --config $1 --steps 3 --warmup 1 > gpurun_out/tr/$1.log 2>&1
python3 - $1 <<'PY'
import csv, sys
r = list(csv.DictReader(open(f'gpurun_out/tr/{sys.argv[1]}/run_kernel_stats.csv')))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:12]:
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>3s} avg_ms={float(x['AverageNs'])/1e6:8.3f}")
PY
