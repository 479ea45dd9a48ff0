#!/bin/bash
# GPU box: direct-path / dev / aligned-group tests, then the integer-dev and
# C3* / 8-way bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_direct.py tests/test_aligned_group.py tests/test_multirank.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_dev.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_dev.log; [ $rc -eq 0 ] || exit $rc
for c in c3_dev_100k c3s; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 5 --warmup 2 --config $c > gpurun_out/q_$c.json 2>gpurun_out/q_$c.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/q_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4))"
done
timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards 8 > gpurun_out/q_r8.json 2>gpurun_out/q_r8.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/q_r8.json').read().strip().splitlines()[-1]);r=d['roofline'];print('r8',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4))"
