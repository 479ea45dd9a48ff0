import sys, os
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/oracle'); sys.path.insert(0, '/root/repo/tests')
import numpy as np
import oracle
from opentsdb_amd import _abi, core, synth
from opentsdb_amd._lib import Context
ctx = Context(0)
ss = synth.regular(300, 3600, _abi.SYN_INT64_COUNTER, seed=11, step=1)
for agg, dsa in [(0, 0), (0, 3), (1, 3)]:
    g = core.run_spanset(ctx, ss, 0, (1 << 32) - 1, agg, False, 60, dsa)
    o = oracle.spangroup(ss, 0, (1 << 32) - 1, agg, False, 60, dsa)
    t = ctx.timing()
    print("agg", agg, "dsa", dsa, "rc", g[0], "err_index", g[5], "n_out", len(g[1]), "oracle", o.code, len(o.ts),
          "paths", t.paths, "n_grid", t.n_grid, flush=True)
    if g[0] == 0 and o.code == 0:
        print(" ts eq", np.array_equal(g[1], o.ts), "bits eq", np.array_equal(g[3], o.bits), g[3][:4], o.bits[:4])
