#!/bin/bash
# GPU box: C2 step time and k_ds_reg time against the uniform E variant's
# waves a span (TSDBHIP_UG_P). Output: gpurun_out/ugp/
set -o pipefail
mkdir -p gpurun_out/ugp
for p in ${PS:-2 4 6 8 12 24}; do
  TSDBHIP_UG_P=$p timeout -k 10 200 python -u bench.py --config c2 --steps 20 --warmup 3 --no-cpu > gpurun_out/ugp/p$p.json 2> gpurun_out/ugp/p$p.err || exit 1
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step'],4), round(r['kernel_ms'],4))" gpurun_out/ugp/p$p.json $p
done
