#!/bin/bash
# GPU box, a round's evidence (part a): the -m gpu suite (short tracebacks
# kept), smoke, the default bench line and the rocprofv3 kernel stats of that
# same command, the 2/4/8-way shard rehearsals (C3*, and C3 rate sum 8-way)
# with the 8-way C3* step trace. Output under gpurun_out/$R/ (R: round tag).
set -o pipefail
R=${R:-r06}
O=gpurun_out/$R; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -x --tb=short -rf --timeout 600 --timeout-method thread -m gpu --durations=15 \
  > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
cat $O/smoke.log
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
cut -c1-300 $O/bench_default.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/benchprof -o run -f csv -- \
  python3 bench.py > $O/bench_under_rocprof.json 2> $O/benchprof.err || exit 1
for n in 2 4 8; do
  timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards $n > $O/rehearse_$n.json 2>$O/rehearse_$n.err || exit 1
  cut -c1-160 $O/rehearse_$n.json
done
timeout -k 10 300 python -u bench.py --config c3r_sum --no-cpu --steps 20 --warmup 3 --rehearse-shards 8 > $O/rehearse_c3r_sum_8.json 2>$O/rehearse_c3r_sum_8.err || exit 1
cut -c1-160 $O/rehearse_c3r_sum_8.json
bash tools/gpu/trace.sh c3s8 k_assemble_tiles --config c3s --rehearse-shards 8 || exit 1
echo evidence_a_done
