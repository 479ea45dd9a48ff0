#!/bin/bash
# reduce chunk-size sweep (spans per chunk target) on C3* and C3
set -e
O=gpurun_out/spc
mkdir -p $O
for c in c3s c3; do for spc in 256 128 64 32; do
  TSDBHIP_SPC=$spc timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu > $O/${c}_$spc.json 2> $O/${c}_$spc.err
  python3 -c "import json; d=json.loads(open('$O/${c}_$spc.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c spc $spc', '%.3f ms' % d['ms_per_step'], 'kernel %.3f device %.3f' % (r['kernel_ms'], r['step_device_ms']))"
done; done
