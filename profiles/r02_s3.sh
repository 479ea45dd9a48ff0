#!/bin/bash
# Round-2 evidence at HEAD (after the pair walk and cached long lerp): full GPU suite, smoke, every config's line with
# its CPU baseline, the default bench + the rocprofv3 kernel stats of that
# same command, PMC passes of C3* (HBM traffic), 2/4/8-way shard rehearsals.
set -e
O=gpurun_out/r02_s3
mkdir -p $O/cfgs
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 120 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
for c in ${CFGS:-c1 c2 c3 c3r_sum c3r_max c3r_dev c3s c3s_gb100 c3s_gb10k c3_gb100 c4 c4i c5 c3_dev_100k}; do
  timeout -k 10 400 python -u bench.py --config $c --steps 10 --warmup 3 --cpu-seconds 8 > $O/cfgs/$c.json 2> $O/cfgs/$c.err
  python3 -c "import json; d=json.loads(open('$O/cfgs/$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$c', '%.3e' % d['value'], '%.3f ms' % d['ms_per_step'], r.get('kernel'), '%.3f' % r.get('kernel_ms', 0))"
done
timeout -k 10 400 python -u bench.py > $O/bench_default.json 2>$O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/benchprof -o run -- python3 bench.py > $O/bench_under_rocprof.json 2>$O/benchprof.err
echo rocprof done
bash profiles/profile.sh c3s --config c3s --steps 3 --warmup 1 > $O/prof_c3s.log 2>&1
cp gpurun_out/prof_c3s/summary.json $O/pmc_c3s.json
echo pmc done
for n in 2 4 8; do
  timeout -k 10 200 python -u bench.py --no-cpu --steps 10 --warmup 3 --rehearse-shards $n > $O/rehearse_$n.json 2> $O/rehearse_$n.err
  python3 -c "import json; d=json.loads(open('$O/rehearse_$n.json').read().strip().splitlines()[-1]); print('rehearse $n', '%.3f ms' % d['ms_per_step'])"
done
