#!/bin/bash
# same-box A/B of two builds (GPU box): libtsdbhip.so vs libtsdbhip_old.so
set -e
mkdir -p gpurun_out/ab3
for i in 1 2; do for v in new old; do
L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/ab3/$v$i.log 2>&1
done; done
python3 profiles/ab_report.py gpurun_out/ab3
