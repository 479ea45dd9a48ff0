#!/bin/bash
# GPU box: an N-way shard rehearsal of one config against several builds of
# the library, 2 alternating runs each. Usage: libs_rehearse.sh <config> <N> lib1.so lib2.so ...
set -o pipefail
c=$1; n=$2; shift 2
for i in 1 2; do for L in "$@"; do
  TSDBHIP_LIB=$PWD/$L timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 3 --no-cpu --rehearse-shards $n > gpurun_out/lr.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open('gpurun_out/lr.json')); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],4), r['kernel'], round(r['kernel_ms'],4))" "$(basename $L) $c x$n"
done; done
