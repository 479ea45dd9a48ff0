#!/bin/bash
# GPU box: tools/gpu/ab.sh over several configs (same box), then the 8-way
# C3* rehearsal A/B. Usage: ab_multi.sh <config>...
set -o pipefail
for c in "$@"; do bash tools/gpu/ab.sh $c || exit 1; done
for v in new old; do
  L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
  TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu --rehearse-shards 8 > gpurun_out/ab_r8_$v.json 2>gpurun_out/ab_r8_$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_r8_$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print('r8 $v',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4))"
done
