#!/bin/bash
set -e
mkdir -p gpurun_out/asm
timeout -k 10 600 python -u -m pytest tests/test_sharded.py tests/test_direct.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/asm/t1.log 2>&1 || { tail -30 gpurun_out/asm/t1.log; exit 1; }
tail -1 gpurun_out/asm/t1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -m gpu -k "assembly or jittered or q1 or short or lazy or empty" > gpurun_out/asm/t2.log 2>&1 || { tail -30 gpurun_out/asm/t2.log; exit 1; }
tail -1 gpurun_out/asm/t2.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/asm/c4 -o run -- python3 bench.py --no-cpu --config c4 --steps 2 --warmup 1 > gpurun_out/asm/c4.log 2>&1
tail -1 gpurun_out/asm/c4.log | cut -c1-200
python3 - <<'PY'
import csv
r = list(csv.DictReader(open('gpurun_out/asm/c4/run_kernel_stats.csv')))
for x in sorted(r, key=lambda x: -float(x['TotalDurationNs']))[:6]:
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>3s} avg_ms={float(x['AverageNs'])/1e6:8.3f}")
PY
