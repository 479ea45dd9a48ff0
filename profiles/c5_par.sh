set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_compaction.py -x -v --timeout 400 --timeout-method thread -m gpu > gpurun_out/c5par.log 2>&1
