#!/bin/bash
# GPU box: rocprofv3 kernel trace + stats of one config's bench (no CPU leg).
# Usage: prof_cfg.sh <config> [extra bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
c=$1; shift
mkdir -p gpurun_out/prof_$c
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run -f csv -- \
  python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu "$@" > gpurun_out/prof_$c/bench.json 2> gpurun_out/prof_$c/bench.err || exit 1
cut -c1-200 gpurun_out/prof_$c/bench.json
