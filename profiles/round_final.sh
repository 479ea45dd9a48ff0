#!/bin/bash
# round-end evidence: full GPU suite, smoke, PMC profiles of C3* and C3, default bench with CPU baseline + its rocprof stats
set -e
mkdir -p gpurun_out/final
timeout -k 10 1000 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/final/pytest.log 2>&1 || { tail -40 gpurun_out/final/pytest.log; exit 1; }
tail -1 gpurun_out/final/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
tail -1 gpurun_out/final/smoke.log
bash profiles/profile.sh c3s --config c3s --steps 3 --warmup 1 > gpurun_out/final/prof_c3s.log 2>&1
bash profiles/profile.sh c3 --config c3 --steps 3 --warmup 1 > gpurun_out/final/prof_c3.log 2>&1
cp gpurun_out/prof_c3s/summary.json profiles/pmc_c3s.json
cp gpurun_out/prof_c3/summary.json profiles/pmc_c3.json
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.log 2>&1
tail -1 gpurun_out/final/bench.log
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/benchprof -o run -- python3 bench.py > gpurun_out/final/benchprof.log 2>&1
echo done
