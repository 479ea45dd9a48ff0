#!/bin/bash
# every BASELINE config through bench.py (GPU box), no CPU baseline
set -e
mkdir -p gpurun_out/cfgs
for c in c1 c2 c3 c3r_sum c3r_max c3r_dev c4 c4i c3s c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/cfgs/$c.log 2>&1 || echo "$c failed"
  python3 -c "import json,sys; d=json.loads(open(\"gpurun_out/cfgs/$c.log\").read().strip().splitlines()[-1]); r=d[\"roofline\"]; print(\"$c\", round(d[\"value\"]/1e9,2), \"Gpts/s\", round(d[\"ms_per_step\"],3), \"ms\", r[\"kernel\"], round(r[\"kernel_ms\"],3), round(r[\"achieved\"]))" || true
done
