#!/bin/bash
# A/B: default vs non-temporal chunk loads (GPU box)
set -e
mkdir -p gpurun_out/ab
for i in 1 2; do
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab/base$i.log 2>&1
TSDBHIP_LIB=$PWD/opentsdb_amd/libtsdbhip_nt.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab/nt$i.log 2>&1
done
python3 profiles/ab_report.py gpurun_out/ab
