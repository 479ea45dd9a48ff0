#!/bin/bash
# Kernel traces of single-GPU config lines (one step's timeline: tools/trace_step.py)
set -o pipefail
O=${1:-gpurun_out/trace_cfgs}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
for c in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 --config $c > $O/$c.json 2> $O/$c.err || exit $?
done
