#!/bin/bash
# GPU box: the given test files first (fail fast), then the whole -m gpu
# suite (HIP runtime errors logged: AMD_LOG_LEVEL=1), then the 8-way shard
# rehearsals (kernel trace of C3*, three unprofiled lines each of C3* and C3
# rate sum) and the default bench line. Logs under gpurun_out/.
set -o pipefail
mkdir -p gpurun_out
FIRST=${FIRST:-tests/test_uniform.py}
timeout -k 10 600 python -u -m pytest $FIRST -q -x --tb=short -rf --timeout 300 --timeout-method thread -m gpu \
  > gpurun_out/pytest_first.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_first.log; [ $rc -eq 0 ] || exit $rc
AMD_LOG_LEVEL=1 timeout -k 10 900 python -u -m pytest tests -q -x --tb=short -rf --timeout 600 --timeout-method thread \
  -m gpu --durations=10 > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu/rehearse8.sh || exit 1
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || exit 1
cut -c1-300 gpurun_out/bench.json
