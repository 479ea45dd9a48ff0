#!/bin/bash
# GPU box: the compaction tests, then C5 per-kernel timings (timing_detail)
# of the library against libtsdbhip_old.so (tools/build_old.sh), same box.
# Usage: c5check.sh [tests|notests]
set -o pipefail
O=gpurun_out/c5check; mkdir -p $O
if [ "${1:-tests}" = tests ]; then
  timeout -k 10 600 python -u -m pytest tests/test_compaction.py -q -x --tb=short -rf --timeout 300 --timeout-method thread -m gpu \
    > $O/pytest.log 2>&1; rc=$?; tail -15 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
for i in 1 2; do for v in new old; do
  L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
  [ -f $L ] || continue
  TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu --option timing_detail=on > $O/$v$i.json 2> $O/$v$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/$v$i.json'));r=d['roofline'];print('$v$i',round(d['ms_per_step'],3),{k:round(v,3) for k,v in r.items() if k.endswith('_ms') and v is not None}, d['config']['status_counts'])"
done; done
