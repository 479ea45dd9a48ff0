#!/bin/bash
# HEAD check (round 2, session 2): full GPU suite, smoke, default bench line
set -e
O=gpurun_out/r02_head
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 400 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for c in c1 c2 c5; do
  timeout -k 10 300 python -u bench.py --config $c --steps 10 --warmup 3 --no-cpu > $O/$c.json 2>$O/$c.err
  tail -1 $O/$c.json | cut -c1-300
done
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2>$O/bench_default.err
tail -1 $O/bench_default.json
