set -o pipefail
mkdir -p gpurun_out
bash tools/gpu/trace.sh c3s8 k_assemble_tiles --config c3s --rehearse-shards 8 || exit 1
for i in 1 2 3; do timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 --config c3s --rehearse-shards 8 > gpurun_out/r8_$i.json || exit 1; timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 --config c3r_sum --rehearse-shards 8 > gpurun_out/r8r_$i.json || exit 1; done
python3 -c "
import json
for p in ['r8_1','r8_2','r8_3','r8r_1','r8r_2','r8r_3']:
    d=json.load(open('gpurun_out/'+p+'.json')); print(p, round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4))"
