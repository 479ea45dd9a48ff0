#!/bin/bash
# GPU box: kernel traces of the small-group step (C1) and of one 8-way shard of C3*.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_c1 gpurun_out/prof_r8
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c1 -o run -f csv -- \
  python3 bench.py --config c1 --steps 50 --warmup 5 --no-cpu > gpurun_out/prof_c1/bench.json 2> gpurun_out/prof_c1/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r8 -o run -f csv -- \
  python3 bench.py --rehearse-shards 8 --steps 20 --warmup 3 --no-cpu > gpurun_out/prof_r8/bench.json 2> gpurun_out/prof_r8/bench.err || exit 1
cut -c1-300 gpurun_out/prof_c1/bench.json gpurun_out/prof_r8/bench.json
find gpurun_out/prof_c1 gpurun_out/prof_r8 -name "*.csv" | head
