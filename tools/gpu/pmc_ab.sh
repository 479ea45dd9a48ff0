#!/bin/bash
# GPU box: HBM fetch / write counters of one config's bench under two values
# of an environment knob. Usage: pmc_ab.sh <config> VAR "v1 v2" [kernel]
set -o pipefail
c=$1; VAR=$2; VALS=$3; K=${4:-k_reduce}
mkdir -p gpurun_out/pmc_ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in $VALS; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    export $VAR=$v
    timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_ab/${c}_${v}_$ctr -o run -- \
      python3 bench.py --no-cpu --steps 3 --warmup 1 --config $c > gpurun_out/pmc_ab/${c}_${v}_$ctr.log 2>&1 || exit 1
    f=$(find gpurun_out/pmc_ab/${c}_${v}_$ctr -name '*counter_collection.csv' | head -1)
    python3 - "$f" "$K" "$VAR=$v $ctr" <<'PY'
import csv, sys
rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"].split("(")[0][-60:], []).append(float(r["Counter_Value"]))
for k, v in by.items():
    print(sys.argv[3], k, "launches", len(v), "avg KB", round(sum(v) / len(v)))
PY
  done
done
