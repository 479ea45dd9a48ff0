#!/bin/bash
# GPU box: one config's bench under several values of a context option
# (bench.py --option NAME=VALUE, tsdbhip_set_option), interleaved twice.
# Usage: ab_env.sh <config> NAME "v1 v2 ..." [extra bench args]
set -o pipefail
c=$1; NAME=$2; VALS=$3; shift 3
mkdir -p gpurun_out/ab
for rep in 1 2; do
  for v in $VALS; do
    timeout -k 10 240 python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu --option $NAME=$v "$@" > gpurun_out/ab/${c}_${v}_$rep.json 2> gpurun_out/ab/${c}_${v}_$rep.err || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/ab/${c}_${v}_$rep.json')); r=d['roofline']; print('$c $NAME=$v rep$rep', round(d['ms_per_step'],3), 'ms', r['kernel'], round(r['kernel_ms'],3), 'frac', round(r['frac'],3))"
  done
done
