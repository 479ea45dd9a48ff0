#!/bin/bash
# GPU box: downsampling parity (GPU tests touching ds / full-size configs), then
# C3*, C2 and the 8-way C3* rehearsal bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_aligned_group.py tests/test_gpu_parity.py tests/test_fullscale.py tests/test_direct.py tests/test_multirank.py tests/test_groupby.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_ds.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ds.log; [ $rc -eq 0 ] || exit $rc
for c in c3s c2; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 3 --config $c > gpurun_out/q_$c.json 2>gpurun_out/q_$c.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/q_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4),'frac',round(r['frac'],3))"
done
timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards 8 > gpurun_out/q_r8.json 2>gpurun_out/q_r8.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/q_r8.json').read().strip().splitlines()[-1]);r=d['roofline'];print('r8',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4),'frac',round(r['frac'],3))"
