#!/bin/bash
# GPU box, a round's evidence (part b): every BASELINE config's bench line
# with its CPU baseline (gpurun_out/$R/cfgs/; tabulated by
# tools/results_table.py).
set -o pipefail
R=${R:-r06}
O=gpurun_out/$R; mkdir -p $O/cfgs
CFGS=${@:-c1 c2 c3 c3r_sum c3r_max c3r_dev c3s c4 c4i c5 c3_dev c3_dev_100k}
for c in $CFGS; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 8 > $O/cfgs/$c.json 2> $O/cfgs/$c.err || exit 1
  python - "$O/cfgs/$c.json" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
r=d.get("roofline",{})
print(sys.argv[1].split('/')[-1], f"{d['value']:.3e}", f"{d['ms_per_step']:.3f}ms", r.get("kernel"), f"{r.get('kernel_ms',0):.3f}ms", f"frac={r.get('frac') or 0:.3f}")
PY
done
echo evidence_b_done
