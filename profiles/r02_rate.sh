#!/bin/bash
# direct-path rate: lane 0 alone loads the previous cell (k_reduce
# direct_run): rate parity, GPU suite, same-box A/B on C3 rate sum / dev
set -e
O=gpurun_out/r02_rate
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -v -x --timeout 60 --timeout-method thread -m gpu -k "rate" > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 60 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu/ab.sh c3r_sum
bash tools/gpu/ab.sh c3r_dev
