#!/bin/bash
# same-box A/B of libtsdbhip.so (new) vs libtsdbhip_old.so, after the GPU suite on the new one
# usage: profiles/ab.sh OUTDIR [bench args...]
set -o pipefail
O=$1; shift
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for i in 1 2 3; do for v in new old; do
L=$PWD/opentsdb_amd/libtsdbhip.so; [ $v = old ] && L=$PWD/opentsdb_amd/libtsdbhip_old.so
TSDBHIP_LIB=$L timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > $O/$v$i.log 2> $O/$v$i.err || exit $?
done; done
python3 profiles/ab_report.py $O
