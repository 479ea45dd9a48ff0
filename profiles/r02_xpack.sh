#!/bin/bash
set -e
O=gpurun_out/r02_xpack
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 --rehearse-shards 8 > $O/rehearse_8.json 2> $O/rehearse_8.err
python3 -c "import json; d=json.loads(open('$O/rehearse_8.json').read().strip().splitlines()[-1]); print('rehearse 8', '%.3f ms' % d['ms_per_step'])"
