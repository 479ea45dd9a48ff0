set -e
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/exp
for v in 0 1; do
  if [ $v = 1 ]; then export TSDBHIP_EXP_NOMARK=1; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/p$v -o run -- python3 bench.py --no-cpu --config c3s --steps 3 --warmup 1 > gpurun_out/exp/p$v.log 2>&1
  grep -h "k_ds_spans\|k_kept\|k_span_sum" gpurun_out/exp/p$v/run_kernel_stats.csv | cut -d, -f1,4 | sed "s/^/v$v /"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM --output-format csv -d gpurun_out/exp/pmc -o run -- python3 bench.py --config c3s --no-cpu --steps 1 --warmup 1 > gpurun_out/exp/pmc.log 2>&1
python3 - <<'PY'
import csv, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open("gpurun_out/exp/pmc/run_counter_collection.csv")):
    if "k_ds_spans" not in r["Kernel_Name"]: continue
    acc[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
for c, d in acc.items(): print(c, sum(d.values()) / len(d))
PY
