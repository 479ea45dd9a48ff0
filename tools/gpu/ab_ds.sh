#!/bin/bash
# GPU box: same-box A/B of the downsampler front (auto: k_ds_reg first; spans:
# k_ds_spans alone) on the given configs, alternating, 3 rounds.
set -o pipefail
mkdir -p gpurun_out
CFGS=${@:-c3s}
for i in 1 2 3; do
  for c in $CFGS; do
    for m in auto spans; do
      if [ $m = auto ]; then unset TSDBHIP_DECODE; else export TSDBHIP_DECODE=$m; fi
      timeout -k 10 300 python -u bench.py --no-cpu --steps 10 --warmup 3 --config $c > gpurun_out/ab_${c}_$m.json 2>gpurun_out/ab_${c}_$m.err || exit 1
      python -c "import json;d=json.loads(open('gpurun_out/ab_${c}_$m.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$i $c $m',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4))"
    done
  done
done
unset TSDBHIP_DECODE
for m in auto spans; do
  if [ $m = auto ]; then unset TSDBHIP_DECODE; else export TSDBHIP_DECODE=$m; fi
  timeout -k 10 300 python -u bench.py --no-cpu --steps 20 --warmup 3 --rehearse-shards 8 > gpurun_out/ab_r8_$m.json 2>gpurun_out/ab_r8_$m.err || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_r8_$m.json').read().strip().splitlines()[-1]);r=d['roofline'];print('r8 $m',round(d['ms_per_step'],4),'kernel_ms',round(r.get('kernel_ms',0),4))"
done
