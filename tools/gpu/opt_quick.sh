#!/bin/bash
# GPU box: multi-rank / aligned-group / parity / full-size tests, then C3*,
# C2 and the 8-way rehearsal lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_multirank.py tests/test_aligned_group.py tests/test_gpu_parity.py tests/test_fullscale.py tests/test_sharded.py tests/test_groupby.py -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest_opt.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_opt.log; [ $rc -eq 0 ] || exit $rc
for c in c3s c2; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 3 --config $c > gpurun_out/q_$c.json 2>gpurun_out/q_$c.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/q_$c.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$c',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4),d.get('paths'))"
done
for n in 8 4; do
timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards $n > gpurun_out/q_r$n.json 2>gpurun_out/q_r$n.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/q_r$n.json').read().strip().splitlines()[-1]);r=d['roofline'];print('r$n',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4),d.get('collectives_per_call'),d.get('paths'))"
done
