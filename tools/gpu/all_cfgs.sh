#!/bin/bash
# GPU box: every bench config with its CPU baseline leg, one JSON line each
# under gpurun_out/all/ (for BASELINE.md's results table).
# Usage: all_cfgs.sh [configs...]
set -o pipefail
mkdir -p gpurun_out/all
CFGS=${@:-c1 c2 c3 c3r_sum c3r_max c3r_dev c3s c3s_gb100 c3s_gb10k c3_gb100 c4 c4i c5}
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 8 \
    > gpurun_out/all/$c.json 2> gpurun_out/all/$c.err || exit 1
  echo "$c done"
done
