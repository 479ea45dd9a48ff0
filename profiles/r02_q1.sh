#!/bin/bash
set -e
O=gpurun_out/r02_q1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -x --timeout 60 --timeout-method thread -m gpu -k "q1" > $O/q1.log 2>&1 || { tail -60 $O/q1.log; exit 1; }
tail -1 $O/q1.log
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 60 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
