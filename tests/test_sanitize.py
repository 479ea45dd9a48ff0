"""The CPU oracle and the host output formatter (fmt.hip) under
AddressSanitizer + UndefinedBehaviorSanitizer (sanitizer
builds of the host code): `make -C oracle sanitize` builds oracle/sanitize.cc
with -fsanitize=address,undefined and runs it over generated SpanGroups
(every aggregator, rate, downsampling, windows, an illegal width), the
sharded full-size oracle, compaction rows of every kind and formatter calls
on edge doubles; any report aborts the run. The GPU library's own host code
is not run under ASan (it needs the GPU; the pool refuses sanitized GPU
runs)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_oracle_and_formatter_clean_under_asan_ubsan():
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True,
                       text=True, timeout=580)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "formatter ok" in r.stdout
