#!/bin/bash
# C4 reduce time split: full / no lerp / no cached-span work (timing-only builds)
set -e
mkdir -p gpurun_out/expc4
for v in libtsdbhip libtsdbhip_nolerp libtsdbhip_nocached; do for c in c4 c4i; do
TSDBHIP_LIB=$PWD/opentsdb_amd/$v.so timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/expc4/$v-$c.log 2>&1
python3 -c "import json; d=json.loads(open('gpurun_out/expc4/$v-$c.log').read().strip().splitlines()[-1]); print('$v $c', round(d['ms_per_step'],2), round(d['roofline']['step_device_ms'],2))"
done; done
