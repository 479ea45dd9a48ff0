#!/bin/bash
# GPU box: one config against several builds of the library (variants built
# here with `make -C opentsdb_amd/csrc OUT=... EXTRA=-D...`), 2 alternating
# runs each. Usage: libs.sh <config> lib1.so lib2.so ... (env BENCH_ARGS:
# extra bench flags, e.g. "--rehearse-shards 8"; TAG: output suffix)
set -o pipefail
c=$1; shift
O=gpurun_out/libs_$c${TAG:+_$TAG}
mkdir -p $O
for i in 1 2; do for L in "$@"; do
  n=$(basename $L .so)
  TSDBHIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu $BENCH_ARGS > $O/$n.$i.json 2> $O/$n.$i.err || exit 1
done; done
python3 - $O <<'PY'
import json, os, sys
d = sys.argv[1]
for f in sorted(os.listdir(d)):
    if f.endswith(".json"):
        j = json.load(open(os.path.join(d, f)))
        r = j["roofline"]
        print(f, round(j["ms_per_step"], 4), {k: round(v, 3) for k, v in r.items() if k.endswith("_ms") and v is not None})
PY
