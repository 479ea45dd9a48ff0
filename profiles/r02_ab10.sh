#!/bin/bash
set -e
O=gpurun_out/r02_ab10
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu/ab.sh c3s --rehearse-shards 8
bash tools/gpu/ab.sh c3s
