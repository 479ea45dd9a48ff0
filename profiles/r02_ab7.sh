#!/bin/bash
set -e
O=gpurun_out/r02_ab7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_compaction.py tests/test_fullscale.py -q -x --timeout 300 --timeout-method thread -m gpu -k "compact" > $O/pytest_c.log 2>&1 || { tail -60 $O/pytest_c.log; exit 1; }
tail -1 $O/pytest_c.log
bash tools/gpu/ab.sh c5
