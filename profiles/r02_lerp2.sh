#!/bin/bash
# one-point-in-tile long lerps from prepared brackets (k_reduce): targeted parity, GPU suite,
# then same-box A/B on C4 / C4-int against the previous build (GPU box)
set -e
O=gpurun_out/r02_lerp2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -v -x --timeout 60 --timeout-method thread -m gpu -k "cached_long_lerp or jittered or minimal_width or known_answers or regular_nods" > $O/t.log 2>&1 || { tail -60 $O/t.log; exit 1; }
tail -1 $O/t.log
timeout -k 10 900 python -u -m pytest tests -q -x --timeout 60 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
bash tools/gpu/ab.sh c4
bash tools/gpu/ab.sh c4i
