#!/bin/bash
# direct path: its tests, the parity suite under TSDBHIP_DECODE=direct, C3 benches, kernel stats
set -e
mkdir -p gpurun_out/dq
timeout -k 10 600 python -u -m pytest tests/test_direct.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/dq/t_direct.log 2>&1 || { tail -30 gpurun_out/dq/t_direct.log; exit 1; }
tail -2 gpurun_out/dq/t_direct.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -m gpu -k "direct" > gpurun_out/dq/t_par.log 2>&1 || { tail -30 gpurun_out/dq/t_par.log; exit 1; }
tail -2 gpurun_out/dq/t_par.log
for c in c3 c3r_sum c3r_dev c1; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/dq/$c.log 2>&1
  python3 -c "import json,sys; d=json.loads(open(\"gpurun_out/dq/$c.log\").read().strip().splitlines()[-1]); r=d[\"roofline\"]; print(\"$c\", round(d[\"value\"]/1e9,2), \"Gpts/s\", round(d[\"ms_per_step\"],3), \"ms\", r[\"kernel\"], round(r[\"kernel_ms\"],3), round(r[\"achieved\"]))"
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dq/prof -o run -- python3 bench.py --no-cpu --config c3r_sum --steps 3 --warmup 1 > gpurun_out/dq/prof.log 2>&1
python3 - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/dq/prof/run_kernel_stats.csv')))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:14]:
    print(f"{x['Name'][:60]:60s} n={x['Calls']:>3s} avg_ms={float(x['AverageNs'])/1e6:8.3f}")
PY
