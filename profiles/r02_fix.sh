#!/bin/bash
set -e
O=gpurun_out/r02_final
mkdir -p $O/cfgs
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for c in ${CFGS:-c1 c4 c4i}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 8 > $O/cfgs/$c.json 2> $O/cfgs/$c.err
  python3 -c "import json; d=json.loads(open('$O/cfgs/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', '%.3e' % d['value'], '%.3f ms' % d['ms_per_step'], r.get('kernel'), '%.3f' % r.get('kernel_ms', 0))"
done
