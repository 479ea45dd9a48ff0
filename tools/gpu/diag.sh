#!/bin/bash
# GPU box: per config, the rocprofv3 kernel stats of a short bench and one
# PMC pass of SQ counters (issue / wait / VMEM). Output: gpurun_out/diag/<c>/
# Usage: diag.sh <config>... (env: BENCH_ARGS for extra bench flags)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in "$@"; do
  O=gpurun_out/diag/$c; mkdir -p $O
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu $BENCH_ARGS > $O/bench.json 2> $O/bench.err || exit 1
  cut -c1-240 $O/bench.json
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU -d $O/pmc_sq -o run -f csv -- \
    python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu $BENCH_ARGS > $O/pmc.log 2>&1 || exit 1
done
python3 tools/diag_summary.py gpurun_out/diag
