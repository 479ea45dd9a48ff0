#!/bin/bash
set -e
mkdir -p gpurun_out/c4q
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded.py -q -x --timeout 300 --timeout-method thread -m gpu -k "jittered or known or ka8 or windows or nan or illegal or mixed" > gpurun_out/c4q/t.log 2>&1 || { tail -30 gpurun_out/c4q/t.log; exit 1; }
tail -1 gpurun_out/c4q/t.log
for c in c4 c4i; do
  timeout -k 10 300 python -u bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/c4q/$c.log 2>&1
  python3 -c "import json,sys; d=json.loads(open(\"gpurun_out/c4q/$c.log\").read().strip().splitlines()[-1]); r=d[\"roofline\"]; print(\"$c\", round(d[\"value\"]/1e9,3), \"Gpts/s\", round(d[\"ms_per_step\"],3), \"ms\", r[\"kernel\"], round(r[\"kernel_ms\"],3), round(r[\"achieved\"]))"
done
