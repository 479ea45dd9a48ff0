#!/bin/bash
# float downsampling in k_ds_spans: parity (chunks + auto paths), C2 bench, C3* A/B vs the previous build
set -e
mkdir -p gpurun_out/dsf
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -q -x --timeout 300 --timeout-method thread -m gpu -k "chunk or auto or regular_ds or sharded" > gpurun_out/dsf/t.log 2>&1 || { tail -30 gpurun_out/dsf/t.log; exit 1; }
tail -1 gpurun_out/dsf/t.log
timeout -k 10 300 python -u bench.py --config c2 --steps 5 --warmup 2 --no-cpu > gpurun_out/dsf/c2.log 2>&1
tail -1 gpurun_out/dsf/c2.log | cut -c 1-120
python3 -c "import json; d=json.loads(open('gpurun_out/dsf/c2.log').read().strip().splitlines()[-1]); r=d['roofline']; print('c2', d['ms_per_step'], r['kernel'], r['kernel_ms'], r['achieved'])"
bash profiles/ab_old_new.sh
