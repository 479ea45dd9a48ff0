"""Debug helper: per-output mismatches of one downsampling case (GPU vs oracle),
and per-span single-series runs to find the spans that differ."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import numpy as np
from helpers import run_both
from opentsdb_amd import _abi, synth, packing
from opentsdb_amd._lib import Context
ctx = Context(0)
ss = synth.regular(30, 2000, _abi.SYN_INT64_COUNTER, seed=5, step=10)
g, o = run_both(ctx, ss, agg=0, ds_interval=60, ds_agg=3)
bad = np.nonzero(g[3] != o.bits)[0]
print("mismatch idx", bad.tolist())
print("gpu", g[3][bad].tolist()); print("ora", o.bits[bad].tolist())
# single-span groups
for s in range(3):
    sub = synth.regular(1, 2000, _abi.SYN_INT64_COUNTER, seed=5, step=10, span0=s)
    g1, o1 = run_both(ctx, sub, agg=0, ds_interval=60, ds_agg=3)
    b1 = np.nonzero(g1[3] != o1.bits)[0]
    print("span", s, "mismatch", b1.tolist(), g1[3][b1].tolist()[:6], o1.bits[b1].tolist()[:6])
