#!/bin/bash
# GPU box: the -m gpu suite (or the given test files), then a short default bench.
set -o pipefail
mkdir -p gpurun_out
ARGS=${@:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -q -x --tb=short -rf --timeout 600 --timeout-method thread -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
cut -c1-600 gpurun_out/bench.json
exit $rc
