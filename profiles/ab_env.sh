#!/bin/bash
# same-box A/B of one build under different values of an experiment variable
# usage: profiles/ab_env.sh OUTDIR VAR "v1 v2 ..." [bench args...]  ("-" = unset)
set -o pipefail
O=$1; VAR=$2; VALS=$3; shift 3
mkdir -p $O
for i in 1 2; do for v in $VALS; do
  if [ "$v" = "-" ]; then env -u $VAR timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > $O/v_def_$i.log 2> $O/v_def_$i.err || exit $?
  else env $VAR=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu "$@" > $O/v_${v}_$i.log 2> $O/v_${v}_$i.err || exit $?; fi
done; done
python3 profiles/ab_report.py $O
