#!/bin/bash
# GPU box: k_ds_reg's duration against the number of series (C3* shape,
# unsharded), to separate size effects (launch tail, ramp) from the sharded
# path's own overhead. Output: gpurun_out/ds_sizes/<n>/
# Usage: ds_reg_sizes.sh <n_series>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for n in "$@"; do
  O=gpurun_out/ds_sizes/$n; mkdir -p $O
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O -o run -f csv -- \
    python3 bench.py --config c3s --series $n --steps 10 --warmup 2 --no-cpu > $O/bench.json 2> $O/bench.err || exit 1
  python3 - "$O" "$n" <<'EOF'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_ds_reg" in r["Name"]:
        print(sys.argv[2], "series: k_ds_reg avg", float(r["AverageNs"]) / 1e3, "us")
EOF
done
