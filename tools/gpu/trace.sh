#!/bin/bash
# GPU box: rocprofv3 kernel trace of one bench command and one step's kernel
# timeline (tools/step_trace.py). Output: gpurun_out/tr/<tag>.*
# Usage: trace.sh <tag> <first kernel of a step> <bench args...>
set -o pipefail
tag=$1; first=$2; shift 2
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tr/$tag -o run -f csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 "$@" > gpurun_out/tr/$tag.json 2> gpurun_out/tr/$tag.err || exit 1
f=$(find gpurun_out/tr/$tag -name '*kernel_trace.csv' | head -1)
python3 tools/step_trace.py $f $first > gpurun_out/tr/$tag.timeline.txt || exit 1
echo "== $tag: $(cut -c1-120 gpurun_out/tr/$tag.json | head -1)"
tail -1 gpurun_out/tr/$tag.timeline.txt
