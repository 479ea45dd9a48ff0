#!/bin/bash
# full GPU suite, then the given bench configs (no CPU baseline)
set -e
mkdir -p gpurun_out/fc
timeout -k 10 1000 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > gpurun_out/fc/pytest.log 2>&1 || { tail -40 gpurun_out/fc/pytest.log; exit 1; }
tail -1 gpurun_out/fc/pytest.log
for c in "$@"; do
  timeout -k 10 300 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/fc/$c.log 2>&1
  python3 -c "import json,sys; d=json.loads(open(\"gpurun_out/fc/$c.log\").read().strip().splitlines()[-1]); r=d[\"roofline\"]; print(\"$c\", round(d[\"value\"]/1e9,3), \"Gpts/s\", round(d[\"ms_per_step\"],3), \"ms\", r[\"kernel\"], round(r[\"kernel_ms\"],3), round(r[\"achieved\"]))"
done
