set -o pipefail
bash tools/gpu/trace.sh c3s8 k_assemble_fast --config c3s --rehearse-shards 8 && \
bash tools/gpu/trace.sh c3s8_noev k_assemble_fast --config c3s --rehearse-shards 8 --option events=none && \
bash tools/gpu/trace.sh c3r8 k_assemble_fast --config c3r_sum --rehearse-shards 8 && \
bash tools/gpu/trace.sh c2 k_assemble --config c2 && \
bash tools/gpu/trace.sh c5 k_compact_quals --config c5 && \
for n in 1 2 3; do timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 --config c3s --rehearse-shards 8 | cut -c1-140; timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 --config c3s --rehearse-shards 8 --option events=none | cut -c1-140; done
