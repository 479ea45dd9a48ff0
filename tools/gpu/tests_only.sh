#!/bin/bash
# GPU box: the given -m gpu test selection (default: the whole suite), log in gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
ARGS=${@:-tests}
timeout -k 10 1000 python -u -m pytest $ARGS -v -x --timeout 600 --timeout-method thread -m gpu --durations=15 \
  > gpurun_out/pytest_sel.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_sel.log
exit $rc
