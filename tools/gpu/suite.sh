#!/bin/bash
# GPU box: the -m gpu suite (or the given pytest args) with durations, log
# under gpurun_out/pytest_gpu.log.
set -o pipefail
mkdir -p gpurun_out
ARGS=${@:-tests}
timeout -k 10 1000 python -u -m pytest $ARGS -q -x --tb=short -rf --timeout 600 --timeout-method thread -m gpu --durations=25 \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
exit $rc
