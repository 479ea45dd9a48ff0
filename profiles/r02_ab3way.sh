#!/bin/bash
# same-box 3-way A/B on C5: libtsdbhip_a.so, libtsdbhip_b.so, libtsdbhip_old.so
set -e
O=gpurun_out/ab3
mkdir -p $O
for i in 1 2; do for v in a b old; do
  TSDBHIP_LIB=$PWD/opentsdb_amd/libtsdbhip_$v.so timeout -k 10 200 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu > $O/$v$i.json 2> $O/$v$i.err
  python3 -c "import json; d=json.loads(open('$O/$v$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v$i', '%.3f' % d['ms_per_step'], 'classify %.3f rows %.3f' % (r['classify_kernel_ms'], r['rows_kernel_ms']))"
done; done
