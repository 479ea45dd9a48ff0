#!/bin/bash
# C5 (row compaction) bench + kernel trace + HBM counters (run on the GPU box).
set -e
mkdir -p gpurun_out/c5
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u bench.py --config c5 --steps 10 --warmup 3 > gpurun_out/c5/bench.log 2>&1
tail -1 gpurun_out/c5/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/trace -o run -- python3 bench.py --config c5 --no-cpu --steps 5 --warmup 1 > gpurun_out/c5/trace.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/c5/pmc_fetch -o run -- python3 bench.py --config c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5/pmc_fetch.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/c5/pmc_write -o run -- python3 bench.py --config c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/c5/pmc_write.log 2>&1
echo c5_done
python3 profiles/pmc_summary.py gpurun_out/c5 c5 > gpurun_out/c5/summary.json
