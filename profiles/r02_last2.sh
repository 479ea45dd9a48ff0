#!/bin/bash
# HEAD check at the end of the session: full GPU suite, smoke, default bench
set -e
O=gpurun_out/r02_last2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2>$O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-250
