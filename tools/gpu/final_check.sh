#!/bin/bash
# GPU box: the full -m gpu suite (short tracebacks kept), smoke, the default
# bench line, then same-box A/Bs against libtsdbhip_old.so on the given configs.
set -o pipefail
O=gpurun_out/final; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -x --tb=short -rf --timeout 600 --timeout-method thread -m gpu \
  > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-200 $O/bench_default.json
for c in "$@"; do bash tools/gpu/ab.sh $c || exit 1; done
