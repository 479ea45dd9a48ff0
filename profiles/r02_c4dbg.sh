#!/bin/bash
set -e
mkdir -p gpurun_out/c4dbg
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4dbg/tr -o run -- python3 bench.py --no-cpu --config c4 --steps 2 --warmup 1 > gpurun_out/c4dbg/tr.log 2>&1
python3 - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/c4dbg/tr/run_kernel_stats.csv')))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:16]:
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>3s} avg_ms={float(x['AverageNs'])/1e6:9.3f}")
PY
