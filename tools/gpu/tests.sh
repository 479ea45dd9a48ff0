#!/bin/bash
# GPU box: the -m gpu suite (or the test files given as arguments), one process.
set -o pipefail
mkdir -p gpurun_out
ARGS=${@:-tests}
timeout -k 10 900 python -u -m pytest $ARGS -q -x --timeout 600 --timeout-method thread -m gpu \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu.log
exit $rc
