#!/bin/bash
set -e
mkdir -p gpurun_out/c5
for m in plain nocomplex c5; do
timeout -k 10 300 python -u bench.py --config c5 --steps 10 --warmup 3 --no-cpu --c5-mix $m > gpurun_out/c5/bench_$m.log 2>&1
python3 -c "import json;d=json.loads(open('gpurun_out/c5/bench_$m.log').read().strip().splitlines()[-1]);print('$m', d['ms_per_step'], d['roofline']['kernel_ms'], d['roofline']['call_achieved'])"
done
