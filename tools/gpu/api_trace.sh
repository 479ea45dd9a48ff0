#!/bin/bash
# GPU box: HIP API + kernel trace of one bench command, one step's host/GPU
# timeline (tools/api_step.py). Usage: api_trace.sh <tag> <first kernel> <bench args...>
set -o pipefail
tag=$1; first=$2; shift 2
mkdir -p gpurun_out/api
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace -d gpurun_out/api/$tag -o run -f csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 "$@" > gpurun_out/api/$tag.json 2> gpurun_out/api/$tag.err || exit 1
python3 tools/api_step.py gpurun_out/api/$tag $first > gpurun_out/api/$tag.txt || exit 1
cat gpurun_out/api/$tag.txt
