#!/bin/bash
# full GPU suite, then the C4 kernel breakdown
set -e
mkdir -p gpurun_out/full
timeout -k 10 1000 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/full/pytest.log 2>&1 || { tail -40 gpurun_out/full/pytest.log; exit 1; }
tail -3 gpurun_out/full/pytest.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/full/c4 -o run -- python3 bench.py --no-cpu --config c4 --steps 2 --warmup 1 > gpurun_out/full/c4.log 2>&1
python3 - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/full/c4/run_kernel_stats.csv')))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:12]:
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>3s} avg_ms={float(x['AverageNs'])/1e6:8.3f}")
PY
