#!/bin/bash
# GPU box: the -m gpu suite after the division-free integer-dev step, then the
# integer-dev lines (100k and 1M series) and C3*.
set -o pipefail
O=gpurun_out/mk; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 600 --timeout-method thread -m gpu \
  > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for c in c3_dev_100k c3_dev c3s; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 --config $c > $O/$c.json 2>$O/$c.err || exit 1
  python -c "import json;d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]);print('$c',round(d['ms_per_step'],4))"
done
echo mk_done
