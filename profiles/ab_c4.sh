#!/bin/bash
# same-box A/B of C4 / C4-int: libtsdbhip.so vs libtsdbhip_old.so (GPU box)
set -e
O=gpurun_out/ab_c4
mkdir -p $O
for i in 1 2; do for v in new old; do for c in c4 c4i; do
L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > $O/${v}_${c}_$i.log 2>&1
done; done; done
python3 profiles/ab_report.py $O
