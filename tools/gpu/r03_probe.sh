#!/bin/bash
# GPU box, round 3: the -m gpu suite (or the given selection), then host-API +
# kernel timelines of one 8-way shard of C3* (rehearsal) and of C1, and the
# rehearsal / default bench lines.
set -o pipefail
mkdir -p gpurun_out
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -q -x --timeout 600 --timeout-method thread \
  -m gpu --durations=20 > gpurun_out/pytest_sel.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_sel.log
[ $rc -eq 0 ] || exit $rc
for n in 8 2; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards $n > gpurun_out/r$n.json 2>gpurun_out/r$n.err || exit 1
  cut -c1-200 gpurun_out/r$n.json; grep -o '"collectives_per_call": [0-9.]*' gpurun_out/r$n.json
done
timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/c3s.json 2>gpurun_out/c3s.err || exit 1
cut -c1-200 gpurun_out/c3s.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/tapi
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/tapi/r8 -o run -f csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 --rehearse-shards 8 > gpurun_out/tapi/r8.json 2> gpurun_out/tapi/r8.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace -d gpurun_out/tapi/c1 -o run -f csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 --config c1 > gpurun_out/tapi/c1.json 2> gpurun_out/tapi/c1.err || exit 1
find gpurun_out/tapi -name '*.csv' | head
