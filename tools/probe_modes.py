"""Achievable-bandwidth probes on the C3* device workload (tsdbhip_bw_probe
modes 0-3), best of 5 each: the ceilings k_ds_spans is compared against."""
import ctypes as C
import json
import sys
import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from opentsdb_amd import _abi, synth  # noqa: E402
from opentsdb_amd._lib import Context  # noqa: E402
from opentsdb_amd._lib import lib  # noqa: E402


def main():
    n_spans = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    ctx = Context(0)
    L = lib()
    d = _abi.SgDesc()
    p = _abi.SynthParams(seed=3, n_spans=n_spans, n_points=3600, t0=synth.T0, step=1,
                         kind=_abi.SYN_INT64_COUNTER, span0=0)
    ctx.check(L.tsdbhip_synth_generate(ctx.handle, C.byref(p), C.byref(d)))
    names = {0: "span_read", 1: "d2d_copy", 2: "flat_read", 3: "span_read_2inflight"}
    res = {}
    for mode in (0, 1, 2, 3, 0, 2):
        ms, nb = C.c_float(), C.c_uint64()
        best = 0.0
        for _ in range(5):
            ctx.check(L.tsdbhip_bw_probe(ctx.handle, C.byref(d), mode, 8, C.byref(ms), C.byref(nb)))
            best = max(best, nb.value / (ms.value * 1e-3) / 1e9)
        res[names[mode]] = max(res.get(names[mode], 0.0), round(best, 1))
        print(names[mode], round(best, 1), "GB/s", flush=True)
    L.tsdbhip_synth_free(ctx.handle, C.byref(d))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
