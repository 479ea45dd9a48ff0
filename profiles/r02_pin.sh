#!/bin/bash
# C4 / C4-int / C3 lines with page-locked result buffers
set -e
O=gpurun_out/r02_pin
mkdir -p $O
for c in c4 c4i c1 c3; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu > $O/$c.json 2> $O/$c.err
  python3 -c "import json; d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', '%.3f ms' % d['ms_per_step'], 'device %.3f kernel %.3f' % (r['step_device_ms'], r['kernel_ms']))"
done
