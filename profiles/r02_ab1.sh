#!/bin/bash
# full GPU suite, then same-box A/B (new vs HEAD build) on C1, C2, C3*
set -e
O=gpurun_out/r02_ab1
mkdir -p $O
TSDBHIP_CHECK_CLEAN=1 timeout -k 10 900 python -u -m pytest tests -v -x --timeout 60 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log; grep -c CHECK_CLEAN $O/pytest_gpu.log || true
for c in c1 c2 c3s; do bash tools/gpu/ab.sh $c; done
