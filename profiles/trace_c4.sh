#!/bin/bash
# C4 / C4-int: bench line + rocprofv3 kernel stats (GPU box)
set -e
O=gpurun_out/c4t
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for c in c4 c4i; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$c -o run -- python3 bench.py --config $c --no-cpu --steps 3 --warmup 1 > $O/$c.json 2>$O/$c.err
tail -1 $O/$c.json
python3 - $O/tr_$c/run_kernel_stats.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:8]:
    print(r["Name"][:70], r["Calls"], "%.3f ms" % (float(r["AverageNs"]) / 1e6))
PY
done
