#!/bin/bash
# GPU box: A/B of the timing-event modes (tsdbhip_set_option "events") on a
# config, alternating arms. Usage: ab_events.sh <config> <rounds> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
c=$1; n=$2; shift 2
for i in $(seq 1 $n); do
  for m in kernel marker none; do
    timeout -k 10 200 python3 bench.py --config $c --no-cpu --option events=$m "$@" > gpurun_out/ab_ev_${c}_$m.$i.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline',{}); print(sys.argv[2], sys.argv[3], round(d['ms_per_step'],4), 'hot', round(r.get('kernel_ms',0),4))" gpurun_out/ab_ev_${c}_$m.$i.json $c $m
  done
done
