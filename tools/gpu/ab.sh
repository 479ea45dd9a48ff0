#!/bin/bash
# GPU box: same-box A/B of opentsdb_amd/libtsdbhip.so (new) against
# libtsdbhip_old.so on one config, 3 alternating runs each.
# Usage: ab.sh <config> [bench args]
set -o pipefail
c=$1; shift
O=gpurun_out/ab_$c
mkdir -p $O
for i in 1 2 3; do for v in new old; do
  L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
  TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu "$@" > $O/$v$i.json 2> $O/$v$i.err || exit 1
done; done
python3 - $O <<'PY'
import json, os, sys
d = sys.argv[1]
for f in sorted(os.listdir(d)):
    if f.endswith(".json"):
        x = json.load(open(os.path.join(d, f)))
        print(f, "kernel_ms", round(x["roofline"]["kernel_ms"], 3), "ms_per_step", round(x["ms_per_step"], 3))
PY
