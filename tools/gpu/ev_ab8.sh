#!/bin/bash
# GPU box: the 8-way C3* shard rehearsal with the timing events carried by
# the launches (default), as markers, and none (A/B of their cost).
set -o pipefail
mkdir -p gpurun_out/evab
for i in 1 2; do
  for ev in kernel marker none; do
    timeout -k 10 120 python3 bench.py --no-cpu --steps 30 --warmup 3 --config c3s --rehearse-shards 8 --option events=$ev > gpurun_out/evab/${ev}_$i.json || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['ms_per_step'],4))" gpurun_out/evab/${ev}_$i.json
  done
done
