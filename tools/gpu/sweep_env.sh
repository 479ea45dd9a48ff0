#!/bin/bash
# GPU box: bench lines over values of one environment knob.
# Usage: sweep_env.sh VAR "v1 v2 ..." "<bench args>" [rounds]
set -o pipefail
VAR=$1; VALS=$2; BARGS=$3; N=${4:-2}
mkdir -p gpurun_out/sweep
for i in $(seq $N); do for v in $VALS; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --no-cpu $BARGS > gpurun_out/sweep/$v.json 2>gpurun_out/sweep/$v.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/sweep/$v.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$i $VAR=$v',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4))"
done; done
