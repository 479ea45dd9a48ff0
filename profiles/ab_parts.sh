#!/bin/bash
# timing-only experiments: which part of the k_ds_spans step costs (results invalid)
set -e
mkdir -p gpurun_out/ab2
for v in base noheads nostage; do
L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v != base ] && L=$PWD/opentsdb_amd/libtsdbhip_$v.so
TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab2/$v.log 2>&1 || true
done
python3 profiles/ab_report.py gpurun_out/ab2
