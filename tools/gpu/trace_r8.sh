#!/bin/bash
# GPU box: kernel + HIP API traces of the 8-way C3* rehearsal and of C3*, one
# step's timeline each (tools/step_trace.py).
set -o pipefail
mkdir -p gpurun_out/tr
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr/r8 -o run -f csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 --rehearse-shards 8 > gpurun_out/tr/r8.json 2> gpurun_out/tr/r8.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tr/c3s -o run -f csv -- \
  python3 bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/tr/c3s.json 2> gpurun_out/tr/c3s.err || exit 1
for n in r8 c3s; do
  f=$(find gpurun_out/tr/$n -name '*kernel_trace.csv' | head -1)
  python3 tools/step_trace.py $f k_assemble_fast > gpurun_out/tr/$n.timeline.txt || exit 1
  cat gpurun_out/tr/$n.timeline.txt
done
