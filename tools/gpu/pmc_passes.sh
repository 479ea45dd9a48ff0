#!/bin/bash
# GPU box: separate rocprofv3 PMC passes (one counter group each, within the
# gfx950 slot limits: 8 SQ, 4 TCC) over a short bench of each config, plus a
# kernel trace. Output: gpurun_out/pmc/<config>/<pass>/.
# Usage: pmc_passes.sh <config>...
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
declare -A P
P[sq_issue]="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
P[sq_lds]="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"
P[fetch]="FETCH_SIZE"
P[write]="WRITE_SIZE"
P[tcc_hit]="TCC_HIT_sum TCC_MISS_sum"
for c in "$@"; do
  O=gpurun_out/pmc/$c; mkdir -p $O
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/trace -o run -f csv -- \
    python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu > $O/trace.log 2>&1 || exit 1
  for p in sq_issue sq_lds fetch write tcc_hit; do
    timeout -s KILL 240 rocprofv3 --pmc ${P[$p]} -d $O/$p -o run -f csv -- \
      python3 bench.py --config $c --steps 2 --warmup 1 --no-cpu > $O/$p.log 2>&1 || exit 1
  done
  echo "$c done"
done
