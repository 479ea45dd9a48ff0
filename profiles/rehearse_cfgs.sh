#!/bin/bash
# 8-way shard rehearsal of the other 1M-series configs (one GPU, 1-rank RCCL
# communicator) beside their N=1 lines, with a kernel trace of each rehearsal.
set -o pipefail
O=${1:-gpurun_out/reh_cfgs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p $O
for c in c3 c3r_sum c3r_dev; do
  timeout -k 10 240 python -u bench.py --no-cpu --steps 10 --warmup 3 --config $c > $O/${c}_n1.json 2> $O/${c}_n1.err || exit $?
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$c -o run -- python3 bench.py --no-cpu --steps 10 --warmup 3 --config $c --rehearse-shards 8 > $O/${c}_r8.json 2> $O/${c}_r8.err || exit $?
done
