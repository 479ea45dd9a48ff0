#!/bin/bash
# GPU box: same-box A/B of opentsdb_amd/libtsdbhip.so (new) against
# libtsdbhip_old.so (tools/build_old.sh) on several configs, 2 alternating
# runs each. Usage: ab_cfgs.sh <config>...  (env STEPS, default 10)
set -o pipefail
O=gpurun_out/ab_cfgs; mkdir -p $O
for c in "$@"; do for i in 1 2; do for v in new old; do
  L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
  [ -f $L ] || continue
  TSDBHIP_LIB=$L timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 3 --no-cpu > $O/$c.$v$i.json 2> $O/$c.$v$i.err || exit 1
  python3 -c "import json;d=json.load(open('$O/$c.$v$i.json'));r=d['roofline'];print('$c $v$i', round(d['ms_per_step'],4), r.get('kernel'), round(r.get('kernel_ms') or 0,4))"
done; done; done
