#!/bin/bash
# GPU box: bench lines of the given configs (no CPU baseline), one JSON each
# under gpurun_out/cfgs/ (suffixed _$TAG when TAG is set). Usage: cfgs.sh c3s c2 c1 ...
set -o pipefail
mkdir -p gpurun_out/cfgs
for c in "$@"; do
  o=$c${TAG:+_$TAG}
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --no-cpu > gpurun_out/cfgs/$o.json 2> gpurun_out/cfgs/$o.err || exit 1
  python - "$o" <<'PY'
import json,sys
d=json.load(open(f"gpurun_out/cfgs/{sys.argv[1]}.json"))
r=d.get("roofline",{})
print(sys.argv[1], f"{d['value']:.3e}", f"{d['ms_per_step']:.3f}ms", r.get("kernel"), f"{r.get('kernel_ms',0):.3f}ms", f"frac={r.get('frac',0):.3f}", "read_frac=", r.get("frac_of_read_stream"))
PY
done
