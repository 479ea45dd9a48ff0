#!/bin/bash
# GPU suite + C3* bench + kernel trace of the bench (GPU box)
set -e
O=gpurun_out/qc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu > $O/c3s.json 2>$O/c3s.err
tail -1 $O/c3s.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu > $O/tr.log 2>&1
echo done
