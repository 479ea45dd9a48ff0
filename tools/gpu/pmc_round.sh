#!/bin/bash
# GPU box: PMC passes + tables for the given configs (profiles/pmc_<config>.json
# candidates under gpurun_out/pmc/). Usage: pmc_r05.sh c3s c2 ...
set -o pipefail
bash tools/gpu/pmc_passes.sh "$@" || exit 1
for c in "$@"; do
  python3 tools/pmc_table.py gpurun_out/pmc/$c r06 > gpurun_out/pmc/pmc_$c.json || exit 1
  python3 tools/pmc_table.py --text gpurun_out/pmc/$c > gpurun_out/pmc/$c/table.txt || exit 1
  head -6 gpurun_out/pmc/$c/table.txt
done
