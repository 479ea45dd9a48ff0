#!/bin/bash
# default bench line (with CPU baseline) and the rocprofv3 kernel stats of the same command
set -o pipefail
O=${1:-gpurun_out/head2}
mkdir -p $O
timeout -k 10 300 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/benchprof -o run -- python3 bench.py > $O/bench_under_rocprof.json 2> $O/benchprof.err || exit $?
