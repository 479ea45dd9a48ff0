#!/bin/bash
# GPU box: one config against several builds of the library (variants built
# here with `make -C opentsdb_amd/csrc OUT=... EXTRA=-D...`), 2 alternating
# runs each. Usage: libs.sh <config> lib1.so lib2.so ...
set -o pipefail
c=$1; shift
O=gpurun_out/libs_$c
mkdir -p $O
for i in 1 2; do for L in "$@"; do
  n=$(basename $L .so)
  TSDBHIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu > $O/$n.$i.json 2> $O/$n.$i.err || exit 1
done; done
python3 - $O <<'PY'
import json, os, sys
d = sys.argv[1]
for f in sorted(os.listdir(d)):
    if f.endswith(".json"):
        r = json.load(open(os.path.join(d, f)))["roofline"]
        print(f, {k: round(v, 3) for k, v in r.items() if k.endswith("_ms")})
PY
