#!/bin/bash
# GPU box: smoke and the default bench line on the shipped build.
set -o pipefail
O=gpurun_out/final; mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-400 $O/bench_default.json
