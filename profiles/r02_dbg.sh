#!/bin/bash
# multirank tests with the zero-on-entry invariant checks on
O=gpurun_out/r02_dbg
mkdir -p $O
TSDBHIP_CHECK_CLEAN=1 timeout -k 10 600 python -u -m pytest tests/test_multirank.py tests/test_sharded.py -v -x --timeout 60 --timeout-method thread -m gpu > $O/pytest.log 2>&1
echo rc=$?
grep -c PASSED $O/pytest.log
grep -m5 "CHECK_CLEAN" $O/pytest.log || true
tail -5 $O/pytest.log
