#!/bin/bash
# GROUP BY batching on the GPU: parity suite of tsdbhip_spangroup_run_batch,
# then the group-by bench lines and the default line with its h2d leg.
set -e
mkdir -p gpurun_out/gb
timeout -k 10 600 python -u -m pytest tests/test_groupby.py tests/test_direct.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/gb/par.log 2>&1
tail -2 gpurun_out/gb/par.log
for c in c3s_gb100 c3s_gb10k c3_gb100 c3 c3s; do
  timeout -k 10 240 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/gb/$c.log 2>&1
  tail -1 gpurun_out/gb/$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', '%.3e'%d['value'], '%.2f ms'%d['ms_per_step'], d['roofline']['kernel'], '%.2f'%d['roofline']['kernel_ms'])"
done
