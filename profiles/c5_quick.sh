#!/bin/bash
# C5 parity + bench + kernel trace (GPU box)
set -e
mkdir -p gpurun_out/c5
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests/test_compaction.py -x -q --timeout 400 --timeout-method thread -m gpu > gpurun_out/c5par.log 2>&1
tail -1 gpurun_out/c5par.log
timeout -k 10 400 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu > gpurun_out/c5/bench.log 2>&1
tail -1 gpurun_out/c5/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/trace -o run -- python3 bench.py --config c5 --no-cpu --steps 5 --warmup 1 > gpurun_out/c5/trace.log 2>&1
grep -i compact gpurun_out/c5/trace/run_kernel_stats.csv | cut -c1-160
