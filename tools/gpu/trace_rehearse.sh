#!/bin/bash
# GPU box: rocprofv3 kernel trace of an N-way shard rehearsal of a config
# (bench.py --rehearse-shards N: rank 0's shard through the sharded path on a
# 1-rank communicator). Usage: trace_rehearse.sh <config> <N>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
c=$1; n=$2
O=gpurun_out/rehearse_${c}_$n; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O -o run -f csv -- \
  python3 bench.py --config $c --steps 20 --warmup 3 --no-cpu --rehearse-shards $n > $O/bench.json 2> $O/bench.err || exit 1
cut -c1-200 $O/bench.json
