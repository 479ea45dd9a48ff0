#!/bin/bash
# GPU box: the compaction GPU tests with the opt-in flat value copy as a third
# path (TSDBHIP_TEST_FLAT=1), then C5 with each value copy, alternating.
set -o pipefail
TSDBHIP_TEST_FLAT=1 timeout -k 10 600 python -u -m pytest tests/test_compaction.py -x -q -m gpu --timeout 300 \
  --timeout-method thread > gpurun_out/flat_tests.log 2>&1; rc=$?; tail -2 gpurun_out/flat_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/ab_opt.sh c5 compact_vals "rows flat"
