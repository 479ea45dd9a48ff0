#!/bin/bash
# C5 grid-cap experiment for k_compact_classify / k_compact_vals
set -e
O=gpurun_out/c5grid
mkdir -p $O
for cap in 65536 8192 4096 2048 1024; do
  TSDBHIP_CQ_GRID_C=$cap TSDBHIP_CQ_GRID_V=$cap timeout -k 10 200 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu > $O/c5_$cap.json 2> $O/c5_$cap.err
  python3 -c "import json; d=json.loads(open('$O/c5_$cap.json').read().strip().splitlines()[-1]); r=d['roofline']; print('cap $cap', '%.3f ms' % d['ms_per_step'], 'copies %.3f classify %.3f rows %.3f' % (r['kernel_ms'], r['classify_kernel_ms'], r['rows_kernel_ms']))"
done
