#!/bin/bash
# same-box A/B of C5 compaction: libtsdbhip.so vs libtsdbhip_old.so (GPU box)
set -e
O=gpurun_out/ab_c5
mkdir -p $O
for i in 1 2; do for v in new old; do for mix in c5 plain; do
L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --config c5 --c5-mix $mix --steps 10 --warmup 3 --no-cpu > $O/${v}_${mix}_$i.log 2>&1
done; done; done
python3 profiles/ab_report.py $O
