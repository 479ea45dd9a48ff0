#!/bin/bash
# refresh: new GPU tests, then the lines of the configs changed since the
# round-2 evidence run (same layout as r02_final.sh)
set -e
O=gpurun_out/r02_final
mkdir -p $O/cfgs
timeout -k 10 300 python -u -m pytest tests/test_timing.py -v -x --timeout 120 --timeout-method thread -m gpu > $O/pytest_timing.log 2>&1 || { tail -60 $O/pytest_timing.log; exit 1; }
tail -1 $O/pytest_timing.log
for c in ${CFGS:-c1 c2 c3r_dev c5}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 8 > $O/cfgs/$c.json 2> $O/cfgs/$c.err
  python3 -c "import json; d=json.loads(open('$O/cfgs/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', '%.3e' % d['value'], '%.3f ms' % d['ms_per_step'], r.get('kernel'), '%.3f' % r.get('kernel_ms', 0))"
done
