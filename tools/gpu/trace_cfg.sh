#!/bin/bash
# GPU box: kernel trace of one config's bench and one step's timeline
# (tools/step_trace.py). Usage: trace_cfg.sh <config> [first kernel of a step]
set -o pipefail
c=$1; first=${2:-k_assemble}
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr/$c -o run -f csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 --config $c > gpurun_out/tr/$c.json 2> gpurun_out/tr/$c.err || exit 1
f=$(find gpurun_out/tr/$c -name '*kernel_trace.csv' | head -1)
python3 tools/step_trace.py $f $first | tee gpurun_out/tr/$c.timeline.txt
