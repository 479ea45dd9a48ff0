#!/bin/bash
set -e
mkdir -p gpurun_out/rw
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -q -x --timeout 120 --timeout-method thread -m gpu > gpurun_out/rw/par.log 2>&1
tail -1 gpurun_out/rw/par.log
for rw in 16384 8192 4096 2048; do TSDBHIP_RW=$rw timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rw/p$rw -o run -- python3 bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/rw/p$rw.log 2>&1; echo rw=$rw; grep -h "k_reduce\|k_finalize\|k_span_summary\|k_decode" gpurun_out/rw/p$rw/run_kernel_stats.csv | cut -d, -f1,4 | cut -c1-90; done
