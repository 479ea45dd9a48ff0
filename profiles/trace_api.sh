#!/bin/bash
# kernel + HIP API + copy timeline of one bench config (no counters):
# trace_api.sh <config> [extra bench args]
set -e
c=$1; shift
mkdir -p gpurun_out/tapi
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/tapi/$c -o run -- python3 bench.py --no-cpu --config $c --steps 20 --warmup 3 "$@" > gpurun_out/tapi/$c.log 2>&1
ls gpurun_out/tapi/$c
