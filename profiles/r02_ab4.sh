#!/bin/bash
# full GPU suite (invariant checks on), smoke, same-box A/B (new vs last commit)
set -e
O=gpurun_out/r02_ab4
mkdir -p $O
TSDBHIP_CHECK_CLEAN=1 timeout -k 10 900 python -u -m pytest tests -v -x --timeout 60 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log; grep -c CHECK_CLEAN $O/pytest_gpu.log || true
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()"
for c in c1 c2 c3 c3s; do bash tools/gpu/ab.sh $c; done
