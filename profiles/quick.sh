#!/bin/bash
# quick GPU iteration: parity suite + C3* bench + kernel-trace stats
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/par.log 2>&1
tail -2 gpurun_out/par.log
timeout -k 10 240 python -u bench.py --config c3s --steps 5 --warmup 2 --no-cpu > gpurun_out/bench.log 2>&1
tail -1 gpurun_out/bench.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/qprof -o run -- python3 bench.py --no-cpu --config c3s --steps 3 --warmup 1 > gpurun_out/qprof.log 2>&1
python3 - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/qprof/run_kernel_stats.csv')))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:14]:
    print(f"{x['Name'][:60]:60s} n={x['Calls']:>3s} avg_ms={float(x['AverageNs'])/1e6:8.3f}")
PY
