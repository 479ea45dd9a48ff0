#!/bin/bash
# Profiling recipe (run on the GPU box from the repo root):
#   kernel trace + stats, then separate PMC passes (one counter group each;
#   MI355X_MICROARCH.md §rocprofv3 PMC slots / §HBM).
# usage: profiles/profile.sh <tag> [bench args...]
set -e
TAG=$1; shift
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --no-cpu "$@" > $OUT/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d $OUT/pmc_sq -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_sq.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/pmc_sq2 -o run -- python3 bench.py --no-cpu "$@" > $OUT/pmc_sq2.log 2>&1
python3 profiles/pmc_summary.py $OUT $TAG > $OUT/summary.json
echo profile_done
