#!/bin/bash
# GPU box: the integer-dev lines (100k and 1M series, no rate) and the
# PCIe-inclusive legs (tools/gpu/h2d.sh).
set -o pipefail
mkdir -p gpurun_out/cfgs
for c in c3_dev_100k c3_dev; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/cfgs/$c.json 2> gpurun_out/cfgs/$c.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[1], round(d['ms_per_step'],3), r['kernel'], round(r['kernel_ms'],3))" gpurun_out/cfgs/$c.json
done
bash tools/gpu/h2d.sh
