set -o pipefail
O=gpurun_out/c5diag; mkdir -p $O
for m in c5 nocomplex plain; do
  timeout -k 10 200 python -u bench.py --config c5 --c5-mix $m --steps 10 --warmup 3 --no-cpu --option timing_detail=on > $O/$m.json 2> $O/$m.err || exit 1
  python3 -c "import json;d=json.load(open('$O/$m.json'));r=d['roofline'];print('$m',round(d['ms_per_step'],3),{k:round(v,3) for k,v in r.items() if k.endswith('_ms') and v is not None}, d['config']['status_counts'])"
done
