#!/bin/bash
set -e
mkdir -p gpurun_out/profc4
for c in c4 c4i; do
TSDBHIP_LIB=$PWD/opentsdb_amd/libtsdbhip_prof.so timeout -k 10 300 python -u bench.py --config $c --steps 1 --warmup 0 --no-cpu > gpurun_out/profc4/$c.log 2>&1
grep PROF gpurun_out/profc4/$c.log | tail -2
done
