#!/bin/bash
# GPU box: the PCIe-inclusive legs (bench.py --h2d) of C3* (100k-series
# sample), C2 and C5, one JSON each under gpurun_out/h2d/.
set -o pipefail
mkdir -p gpurun_out/h2d
for c in c3s c2 c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu --h2d > gpurun_out/h2d/h2d_$c.json 2> gpurun_out/h2d/h2d_$c.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); h=d['h2d']; print(sys.argv[1], round(d['ms_per_step'],3), {k: (round(v,3) if isinstance(v,float) else v) for k,v in h.items() if k!='sample'})" gpurun_out/h2d/h2d_$c.json
done
