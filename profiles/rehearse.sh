#!/bin/bash
# Shard rehearsal: per-rank work of an N-GPU C3* run on one GPU (1-rank RCCL
# communicator, TSDBHIP_SHARDED), plus a rocprofv3 kernel trace of the 8-way shard.
# usage: profiles/rehearse.sh [outdir] [extra bench args...]
set -o pipefail
O=${1:-gpurun_out/rehearse}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_sharded.py > $O/pytest_sharded.log 2>&1 || exit $?
timeout -k 10 240 python -u bench.py --no-cpu --steps 10 --warmup 3 "$@" > $O/n1.json 2> $O/n1.err || exit $?
for n in 2 4 8; do
  timeout -k 10 180 python -u bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards $n "$@" > $O/r$n.json 2> $O/r$n.err || exit $?
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof8 -o run -- python3 bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards 8 "$@" > $O/prof8.json 2> $O/prof8.err || exit $?
tail -2 $O/pytest_sharded.log
