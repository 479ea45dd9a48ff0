#!/bin/bash
# GPU box: same-box A/B (libtsdbhip.so vs libtsdbhip_old.so) of the N-way
# shard rehearsal, 4 alternating runs each. Usage: ab_r8.sh [N]
set -o pipefail
N=${1:-8}
mkdir -p gpurun_out/abr
for i in 1 2 3 4; do for v in new old; do
  L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
  TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu --rehearse-shards $N > gpurun_out/abr/$v$i.json 2>gpurun_out/abr/$v$i.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abr/$v$i.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$i $v',round(d['ms_per_step'],4),'dev',round(r['step_device_ms'],4),'kernel',round(r.get('kernel_ms',0),4))"
done; done
