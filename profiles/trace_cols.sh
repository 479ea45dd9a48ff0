#!/bin/bash
# kernel traces of C3 at N=1 and as an 8-way shard rehearsal (chunk merge kernels)
set -o pipefail
O=gpurun_out/trace_cols
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/n1 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 --config c3 > $O/n1.json 2> $O/n1.err || exit $?
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r8 -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 --config c3 --rehearse-shards 8 > $O/r8.json 2> $O/r8.err || exit $?
