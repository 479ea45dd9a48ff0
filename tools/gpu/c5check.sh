#!/bin/bash
# GPU box: the compaction tests, then C5 per-kernel timings of the default
# path and the split path (timing_detail), same box.
set -o pipefail
O=gpurun_out/c5check; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_compaction.py -q -x --tb=short -rf --timeout 600 --timeout-method thread -m gpu \
  > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
for p in auto split; do
  timeout -k 10 200 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu --option timing_detail=on --option compact=$p > $O/$p.json 2> $O/$p.err || exit 1
  python3 -c "import json;d=json.load(open('$O/$p.json'));r=d['roofline'];print('$p',round(d['ms_per_step'],3),{k:round(v,3) for k,v in r.items() if k.endswith('_ms') and v is not None}, d['config']['status_counts'])"
done
