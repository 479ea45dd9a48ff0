"""Host cost of hipEventElapsedTime / hipEventQuery on completed events (GPU box).
python3 tools/gpu/ev_cost.py"""
import ctypes as C
import time

hip = C.CDLL("libamdhip64.so")
ev = [C.c_void_p() for _ in range(4)]
for e in ev:
    assert hip.hipEventCreate(C.byref(e)) == 0
hip.hipSetDevice(0)
for e in ev:
    assert hip.hipEventRecord(e, None) == 0
assert hip.hipDeviceSynchronize() == 0
ms = C.c_float()
n = 2000
t0 = time.perf_counter()
for _ in range(n):
    hip.hipEventElapsedTime(C.byref(ms), ev[0], ev[1])
t1 = time.perf_counter()
for _ in range(n):
    hip.hipEventQuery(ev[1])
t2 = time.perf_counter()
for _ in range(n):
    hip.hipEventRecord(ev[2], None)
hip.hipDeviceSynchronize()
t3 = time.perf_counter()
t4 = time.perf_counter()
for _ in range(n):
    hip.hipGetLastError()
t5 = time.perf_counter()
nf = C.c_void_p()
assert hip.hipEventCreateWithFlags(C.byref(nf), 0x20000000) == 0  # hipEventDisableSystemFence
t6 = time.perf_counter()
for _ in range(n):
    hip.hipEventRecord(nf, None)
hip.hipDeviceSynchronize()
t7 = time.perf_counter()
print(f"hipEventRecord (no system fence) {(t7 - t6) / n * 1e6:.2f} us")
print(f"hipEventElapsedTime {(t1 - t0) / n * 1e6:.2f} us, hipEventQuery {(t2 - t1) / n * 1e6:.2f} us, "
      f"hipEventRecord {(t3 - t2) / n * 1e6:.2f} us, ctypes call floor {(t5 - t4) / n * 1e6:.2f} us")
