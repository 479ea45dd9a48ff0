#!/bin/bash
# round-end evidence (session 5): full GPU suite, smoke, every config's bench
# line (incl. GROUP BY and the PCIe-inclusive h2d leg), PMC profiles of C3*
# and C3, the default bench with CPU baseline and the rocprof stats of that
# same command. Everything lands in gpurun_out/final4 (copied to profiles/).
set -e
O=gpurun_out/final4
mkdir -p $O/cfgs
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for c in c1 c2 c3 c3r_sum c3r_max c3r_dev c4 c4i c3s c3s_gb100 c3s_gb10k c3_gb100 c5; do
  timeout -k 10 400 python -u bench.py --config $c --steps 5 --warmup 2 --no-cpu > $O/cfgs/$c.json 2>$O/cfgs/$c.err
  python3 -c "import json; d=json.loads(open('$O/cfgs/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', '%.3e' % d['value'], '%.3f ms' % d['ms_per_step'], r['kernel'], '%.3f' % r['kernel_ms'])"
done
timeout -k 10 400 python -u bench.py --config c3s --steps 3 --warmup 1 --no-cpu --h2d > $O/cfgs/c3s_h2d.json 2>&1
bash profiles/profile.sh c3s --config c3s --steps 3 --warmup 1 > $O/prof_c3s.log 2>&1
bash profiles/profile.sh c3 --config c3 --steps 3 --warmup 1 > $O/prof_c3.log 2>&1
cp gpurun_out/prof_c3s/summary.json $O/pmc_c3s.json
cp gpurun_out/prof_c3/summary.json $O/pmc_c3.json
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2>$O/bench_default.err
tail -1 $O/bench_default.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/benchprof -o run -- python3 bench.py > $O/bench_under_rocprof.json 2>$O/benchprof.err
echo done
# 2/4/8-way shard rehearsals of the default line (per-rank work + exchange code)
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 --rehearse-shards $n > gpurun_out/final4/rehearse_$n.json 2> gpurun_out/final4/rehearse_$n.err
done
echo rehearsals done
