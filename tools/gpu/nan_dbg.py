import sys
import os; R = os.environ.get("GRAFT_REPO_ROOT", "/root/repo"); sys.path[:0] = [R, R + "/tests", R + "/oracle"]
from test_double_sums import groups_list
from helpers import F, T0, U32MAX
from opentsdb_amd import _abi, core, packing
from opentsdb_amd._lib import Context
ctx = Context(0)
spans = [F([(T0 + 7 * i + 3, float("nan") if i == 60_000 else 1.5) for i in range(100_000)], double=True)]
ss = packing.pack_spans(groups_list(3) + spans)
g = core.run_spanset(ctx, ss, 0, U32MAX, _abi.AGG_SUM)
print("rc", g[0], "err", ctx.last_error() if hasattr(ctx, "last_error") else None)
# the suite's order: test_opposite_slopes_line_in_t's calls first, on the same context
from test_double_sums import groups
for seed in (1, 2):
    for agg in (_abi.AGG_SUM, _abi.AGG_AVG):
        s2 = groups(seed)
        for kw in ({}, {"register_out": True}, {"exact": True}):
            g = core.run_spanset(ctx, s2, 0, U32MAX, agg, **kw)
            print(seed, agg, kw, "rc", g[0], ctx.last_error() if g[0] else "")
for reg in (False, True):
    g = core.run_spanset(ctx, ss, 0, U32MAX, _abi.AGG_SUM, register_out=reg)
    print("nan", reg, "rc", g[0], ctx.last_error())
