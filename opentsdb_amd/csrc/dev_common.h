// dev_common.h — device helpers shared by the tsdbhip kernels (gfx950, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define WAVE 64
#define DEVI __device__ __forceinline__

namespace tsdb {

// ---- Java `long` / `double` semantics ------------------------------------
DEVI int64_t ladd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
DEVI int64_t lsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }
DEVI int64_t lmul(int64_t a, int64_t b) { return (int64_t)((uint64_t)a * (uint64_t)b); }
// Java truncating division; MIN/-1 = MIN (no trap).
DEVI int64_t ldiv(int64_t a, int64_t b) {
  if (b == -1) return (int64_t)(0 - (uint64_t)a);
  return a / b;
}
// Java (long)double: NaN -> 0, saturating.
DEVI int64_t d2l(double d) {
  if (d != d) return 0;
  if (d >= 9223372036854775807.0) return INT64_MAX;
  if (d <= -9223372036854775808.0) return INT64_MIN;
  return (int64_t)d;
}
DEVI double bitsd(int64_t b) { return __longlong_as_double(b); }
DEVI int64_t dbits(double d) { return __double_as_longlong(d); }

// ---- errors: the first in the reference's evaluation order wins ----------
// key = stage | order within the stage | -code, reduced with atomicMin (and
// the same MIN across ranks). Stages: 0 Span.addRow while TsdbQuery.findSpans
// scans rows (row-key order: base time, then span), 1 SpanGroup.add in span
// order (TsdbQuery.java:301-307), 2 iteration.
#define ERR_NONE (~0ull)

// The speculative aligned group's condition, read from the call state as the
// host would read it (uniform_run's "fits"): no error, every kept span
// proposed one integer key of >= 64 cells, at most 64 buckets a span.
// (the host decides with the same function from the published state)
__host__ __device__ inline bool ug_spec_fits(unsigned long long k0, unsigned long long k1, unsigned long long k2,
                                             unsigned long long k3, uint64_t n_kept, unsigned long long err,
                                             int64_t interval, uint32_t* nb_out = nullptr, uint32_t* kk_out = nullptr) {
  if (!(err == ERR_NONE && n_kept > 0 && k0 != ~0ull && k0 == k1 && k2 == k3 && (uint32_t)k0 >= 64 && !(k2 & 8u) &&
        interval > 0))
    return false;
  const uint64_t step = k2 >> 32, n = (uint32_t)k0;
  if (step == 0) return false;
  const uint64_t kk = ((uint64_t)interval + step - 1) / step, nb = (n + kk - 1) / kk;
  if (nb_out) *nb_out = (uint32_t)nb;
  if (kk_out) *kk_out = (uint32_t)kk;
  return nb <= WAVE;
}
DEVI void err_raise(unsigned long long* e, uint32_t stage, uint64_t order, int code) {
  atomicMin(e, ((unsigned long long)stage << 62) | ((order & ((1ull << 54) - 1)) << 8) |
                   (unsigned long long)(uint8_t)(-code));
}
DEVI uint64_t err_scan_order(uint32_t base_time, uint32_t span) {
  return ((uint64_t)base_time << 22) | (span < (1u << 22) ? span : (1u << 22) - 1);
}

// ---- wave helpers ----------------------------------------------------------
DEVI int lane_id() { return __lane_id(); }
DEVI uint64_t ballot(bool p) { return __ballot(p); }
DEVI uint64_t lanemask_le(int lane) { return lane == 63 ? ~0ull : ((2ull << lane) - 1); }
DEVI uint64_t lanemask_lt(int lane) { return (1ull << lane) - 1; }

// ---- DPP wave scans (row_shr within 16-lane rows, then row_bcast 15/31) ----
// Pure VALU: no LDS traffic, unlike __shfl (ds_bpermute).
template <int CTRL, int ROWMASK>
DEVI uint32_t dpp_u32(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xf, false);
}
DEVI uint32_t wave_incl_scan_u32_dpp(uint32_t x) {
  x += dpp_u32<0x111, 0xf>(x);
  x += dpp_u32<0x112, 0xf>(x);
  x += dpp_u32<0x114, 0xf>(x);
  x += dpp_u32<0x118, 0xf>(x);
  x += dpp_u32<0x142, 0xa>(x);
  x += dpp_u32<0x143, 0xc>(x);
  return x;
}
// the wave's maximum of non-negative x (DPP max scan; lanes outside a step's
// source keep 0, the identity), uniform
DEVI uint32_t wave_max_u32_dpp(uint32_t x) {
  x = max(x, dpp_u32<0x111, 0xf>(x));
  x = max(x, dpp_u32<0x112, 0xf>(x));
  x = max(x, dpp_u32<0x114, 0xf>(x));
  x = max(x, dpp_u32<0x118, 0xf>(x));
  x = max(x, dpp_u32<0x142, 0xa>(x));
  x = max(x, dpp_u32<0x143, 0xc>(x));
  return __builtin_amdgcn_readlane(x, 63);
}
template <int CTRL, int ROWMASK>
DEVI uint64_t dpp_u64(uint64_t x) {
  const uint32_t lo = dpp_u32<CTRL, ROWMASK>((uint32_t)x);
  const uint32_t hi = dpp_u32<CTRL, ROWMASK>((uint32_t)(x >> 32));
  return ((uint64_t)hi << 32) | lo;
}
// 64-bit inclusive wave scan: each DPP step is one add-with-carry pair
// (lanes whose DPP source is out of range, or whose row is masked off, keep
// their value: bound_ctrl off, so neither half is written there).
DEVI uint64_t wave_incl_scan_u64_dpp(uint64_t x) {
  uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  asm volatile(
      "s_nop 1\n"
      "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf\n"
      "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:1 row_mask:0xf bank_mask:0xf\n"
      "s_nop 1\n"
      "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf\n"
      "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:2 row_mask:0xf bank_mask:0xf\n"
      "s_nop 1\n"
      "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf\n"
      "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:4 row_mask:0xf bank_mask:0xf\n"
      "s_nop 1\n"
      "v_add_co_u32_dpp %0, vcc, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf\n"
      "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_shr:8 row_mask:0xf bank_mask:0xf\n"
      "s_nop 1\n"
      "v_add_co_u32_dpp %0, vcc, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n"
      "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_bcast:15 row_mask:0xa bank_mask:0xf\n"
      "s_nop 1\n"
      "v_add_co_u32_dpp %0, vcc, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n"
      "v_addc_co_u32_dpp %1, vcc, %1, %1, vcc row_bcast:31 row_mask:0xc bank_mask:0xf\n"
      "s_nop 1\n"
      : "+v"(lo), "+v"(hi)
      :
      : "vcc");
  return ((uint64_t)hi << 32) | lo;
}

// floor(a / n) for u64 a, u32 n > 0 — the general case, out of line.
__device__ __attribute__((noinline)) uint64_t udiv64_32_slow(uint64_t a, uint32_t n) {
  if (n <= 1) return n ? a : 0;  // (n == 0 only on a discarded lane: no loop)
  uint64_t q = (uint64_t)((double)a / (double)n);
  int64_t r = (int64_t)(a - q * (uint64_t)n);
  q += (int64_t)floor((double)r / (double)n);
  r = (int64_t)(a - q * (uint64_t)n);
  while (r < 0) { q--; r += n; }
  while (r >= (int64_t)n) { q++; r -= n; }
  return q;
}
// floor(a / n): 32-bit path, or for a < 2^52 a refined double reciprocal
// (error < 1) plus one exact correction step; larger a out of line.
DEVI uint64_t udiv64_32(uint64_t a, uint32_t n) {
  if ((a >> 32) == 0) return (uint32_t)a / n;
  if ((a >> 52) != 0) return udiv64_32_slow(a, n);
  const double dn = (double)n;
  double r = __builtin_amdgcn_rcp(dn);
  r = __builtin_fma(r, __builtin_fma(-dn, r, 1.0), r);  // one Newton step
  uint64_t q = (uint64_t)__builtin_floor((double)a * r);
  const int64_t rem = (int64_t)(a - q * (uint64_t)n);
  if (rem < 0) q--;
  else if (rem >= (int64_t)n) q++;
  return q;
}
// Java long / int with truncation toward zero (n >= 1).
DEVI int64_t ldiv64_32(int64_t a, uint32_t n) {
  if (a >= INT32_MIN && a <= INT32_MAX && n <= (uint32_t)INT32_MAX) return (int64_t)((int32_t)a / (int32_t)n);
  const uint64_t ua = a < 0 ? (uint64_t)0 - (uint64_t)a : (uint64_t)a;
  const uint64_t q = udiv64_32(ua, n);
  return a < 0 ? (int64_t)((uint64_t)0 - q) : (int64_t)q;
}

// Lanes of one wave exchanging data through LDS: the wave's LDS operations
// execute in order, so only the compiler must not move accesses across.
DEVI void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Host-visible publish of a small device state (a call's host round trip
// without a copy and a stream sync): one wave copies nwords 8-byte words of
// src (device-coherent loads) into mapped pinned host memory, fences at
// system scope, then lane 0 stores `seq` to the flag the host spins on.
// Vector stores only. Call from one whole wave after the state is final.
struct HostPub {
  uint64_t* dst;   // mapped host words (device pointer), null: no publish
  uint64_t* flag;  // mapped host flag
  uint64_t seq;
  uint32_t nwords;
};
DEVI void host_publish(const HostPub& p, const uint64_t* src) {
  const int lane = threadIdx.x & (WAVE - 1);
  for (uint32_t i = lane; i < p.nwords; i += WAVE) {
    const uint64_t v = __hip_atomic_load(src + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(p.dst + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) __hip_atomic_store(p.flag, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Position of the (j+1)-th set bit of m (j per lane); requires j < popc(m).
DEVI int select_bit(uint64_t m, int j) {
  int p = 0;
#pragma unroll
  for (int step = 32; step > 0; step >>= 1) {
    const uint64_t low = m & ((1ull << (p + step)) - 1);
    if (__popcll(low) <= j) p += step;
  }
  return p;
}

DEVI uint32_t readlane_u32(uint32_t v, int l) { return __builtin_amdgcn_readlane(v, l); }
DEVI uint64_t readlane_u64(uint64_t v, int l) {
  uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, l);
  uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), l);
  return ((uint64_t)hi << 32) | lo;
}
DEVI uint32_t shfl_u32(uint32_t v, int src) { return __shfl(v, src); }
DEVI uint64_t shfl_u64(uint64_t v, int src) {
  uint32_t lo = __shfl((uint32_t)v, src), hi = __shfl((uint32_t)(v >> 32), src);
  return ((uint64_t)hi << 32) | lo;
}
DEVI uint32_t shfl_up_u32(uint32_t v, int d) { return __shfl_up(v, d); }
// lane l gets lane l-1's x; lane 0 gets `old` (DPP wave_shr:1, gfx9 family)
DEVI uint64_t wave_shr1_u64(uint64_t x, uint64_t old) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)x, 0x138, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(old >> 32), (int)(uint32_t)(x >> 32), 0x138,
                                                            0xF, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}
// lane l gets lane l+1's x; lane 63 gets `old` (DPP wave_shl:1)
DEVI uint64_t wave_shl1_u64(uint64_t x, uint64_t old) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)old, (int)(uint32_t)x, 0x130, 0xF, 0xF, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp((int)(uint32_t)(old >> 32), (int)(uint32_t)(x >> 32), 0x130,
                                                            0xF, 0xF, false);
  return ((uint64_t)hi << 32) | lo;
}
DEVI uint64_t shfl_up_u64(uint64_t v, int d) {
  uint32_t lo = __shfl_up((uint32_t)v, d), hi = __shfl_up((uint32_t)(v >> 32), d);
  return ((uint64_t)hi << 32) | lo;
}
DEVI uint64_t shfl_xor_u64(uint64_t v, int m) {
  uint32_t lo = __shfl_xor((uint32_t)v, m), hi = __shfl_xor((uint32_t)(v >> 32), m);
  return ((uint64_t)hi << 32) | lo;
}

// Inclusive wave scan (wrapping add).
DEVI uint64_t wave_incl_scan_u64(uint64_t x) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint64_t y = shfl_up_u64(x, d);
    if (l >= d) x += y;
  }
  return x;
}
DEVI uint32_t wave_incl_scan_u32(uint32_t x) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = shfl_up_u32(x, d);
    if (l >= d) x += y;
  }
  return x;
}
// Segmented inclusive scan: `head` marks lanes that start a segment.
DEVI uint32_t wave_seg_scan_u32(uint32_t x, uint64_t head_mask) {
  const int l = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t y = shfl_up_u32(x, d);
    // lanes (l-d, l] contain no head -> same segment
    uint64_t win = (l >= d) ? (lanemask_le(l) & ~lanemask_le(l - d)) : 0;
    if (l >= d && (head_mask & win) == 0) x += y;
  }
  return x;
}
DEVI uint64_t wave_or_u64(uint64_t x) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) x |= shfl_xor_u64(x, m);
  return x;
}
DEVI uint64_t wave_sum_u64(uint64_t x) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) x += shfl_xor_u64(x, m);
  return x;
}
DEVI int64_t wave_min_i64(int64_t x) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) { int64_t y = (int64_t)shfl_xor_u64((uint64_t)x, m); x = y < x ? y : x; }
  return x;
}
DEVI int64_t wave_max_i64(int64_t x) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) { int64_t y = (int64_t)shfl_xor_u64((uint64_t)x, m); x = y > x ? y : x; }
  return x;
}

// Block-level (256 threads) combine of one 64-bit value per thread; the
// result is valid in thread 0. Few atomics per launch: same-address atomics
// serialise at one L2 channel (~10 ns each).
template <typename T, typename F>
DEVI T block_reduce_256(T x, F op, T* sh /* [4] */) {
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    T y;
    if (sizeof(T) == 8) y = (T)shfl_xor_u64((uint64_t)x, m);
    else y = (T)__shfl_xor((int)x, m);
    x = op(x, y);
  }
  __syncthreads();
  if (lane_id() == 0) sh[threadIdx.x / 64] = x;
  __syncthreads();
  if (threadIdx.x == 0) x = op(op(sh[0], sh[1]), op(sh[2], sh[3]));
  return x;
}

// ---- big-endian cell decoding (org.hbase.async.Bytes, restated) -----------
DEVI uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }
DEVI uint64_t bswap64(uint64_t x) { return __builtin_bswap64(x); }

// 2-byte big-endian qualifier at an even byte offset.
DEVI uint32_t load_qual(const uint8_t* q, uint64_t off) {
  uint16_t v = *(const uint16_t*)(q + off);
  return (uint32_t)(((v & 0xFF) << 8) | (v >> 8));
}

// Loads `len` (1..8) bytes at arbitrary byte offset `off` as a big-endian
// unsigned number. The buffer must have >= 12 readable bytes past any value.
DEVI uint64_t load_be_bytes(const uint8_t* base, uint64_t off, int len) {
  uint64_t raw;
  if (len == 8 && (off & 7) == 0) {
    raw = *(const uint64_t*)(base + off);
  } else if (len == 4 && (off & 3) == 0) {
    raw = *(const uint32_t*)(base + off);
  } else {
    const uint64_t a = off & ~3ull;
    const int sh = (int)(off & 3) * 8;
    const uint32_t* p = (const uint32_t*)(base + a);
    uint32_t d0 = p[0], d1 = p[1], d2 = (sh + len * 8 > 64) ? p[2] : 0u;
    uint64_t lo = (uint64_t)d0 | ((uint64_t)d1 << 32);
    raw = sh ? ((lo >> sh) | ((uint64_t)d2 << (64 - sh))) : lo;
  }
  // raw holds bytes b0..b7 little-endian; take len bytes, reverse.
  const uint64_t be = bswap64(raw);       // b0 in the top byte
  return be >> (64 - 8 * len);            // b0..b(len-1) as BE number
}

// Decodes one cell value per RowSeq.extractIntegerValue /
// extractFloatingPointValue (RowSeq.java:194-226). Returns false on an
// IllegalDataException width. `bits` receives the long, or the double bits
// (float32 widened exactly).
DEVI bool decode_value(const uint8_t* vals, uint64_t off, uint32_t flags, int64_t* bits) {
  const int lm = flags & 7;
  const int len = lm + 1;
  if (flags & 8) {
    if (lm == 7) { *bits = (int64_t)load_be_bytes(vals, off, 8); return true; }
    if (lm == 3) {
      uint32_t u = (uint32_t)load_be_bytes(vals, off, 4);
      *bits = dbits((double)__uint_as_float(u));
      return true;
    }
    *bits = 0;
    return false;
  }
  if (lm == 7 || lm == 3 || lm == 1 || lm == 0) {
    uint64_t u = load_be_bytes(vals, off, len);
    const int sh = 64 - 8 * len;
    *bits = (int64_t)(u << sh) >> sh;  // sign-extend
    return true;
  }
  *bits = 0;
  return false;
}

// decode_value of a value already assembled: u = its bytes, big-endian, in
// the low bits (len = (flags & 7) + 1 bytes)
DEVI bool decode_be(uint64_t u, uint32_t flags, int64_t* bits) {
  const int lm = flags & 7;
  if (flags & 8) {
    if (lm == 7) { *bits = (int64_t)u; return true; }
    if (lm == 3) { *bits = dbits((double)__uint_as_float((uint32_t)u)); return true; }
    *bits = 0;
    return false;
  }
  if (lm == 7 || lm == 3 || lm == 1 || lm == 0) {
    const int sh = 64 - 8 * (lm + 1);
    *bits = (int64_t)(u << sh) >> sh;  // sign-extend
    return true;
  }
  *bits = 0;
  return false;
}

// toDouble() of a decoded cell / E point.
DEVI double to_double(int64_t bits, bool is_float) { return is_float ? bitsd(bits) : (double)bits; }

// ---- Welford state per Aggregators.StdDev (Aggregators.java:196-238) ------
struct Welford {
  int64_t n;      // values seen
  double mean;
  double var;     // running M2
};
DEVI void wf_init(Welford& w) { w.n = 0; w.mean = 0; w.var = 0; }
DEVI void wf_push(Welford& w, double x) {
  if (w.n == 0) { w.mean = x; w.n = 1; return; }
  w.n++;
  const double nm = w.mean + (x - w.mean) / (double)w.n;
  w.var += (x - w.mean) * (x - nm);
  w.mean = nm;
}
// The same with (x - mean) / n as a product with a refined reciprocal of n
// (within an ulp or two of the quotient): for double-path dev outside
// TSDBHIP_EXACT_ORDER, whose tolerance (1e-9 relative) already admits the
// chunk-merge reordering; integer dev and EXACT_ORDER keep the division.
DEVI void wf_push_rcp(Welford& w, double x) {
  if (w.n == 0) { w.mean = x; w.n = 1; return; }
  w.n++;
  const double dn = (double)w.n;
  double r = __builtin_amdgcn_rcp(dn);
  r = __builtin_fma(__builtin_fma(-dn, r, 1.0), r, r);  // one Newton step
  const double d = x - w.mean;
  const double nm = __builtin_fma(d, r, w.mean);
  w.var += d * (x - nm);
  w.mean = nm;
}
// Chan et al. merge (A precedes B); used only across span chunks/ranks.
DEVI void wf_merge(Welford& a, const Welford& b) {
  if (b.n == 0) return;
  if (a.n == 0) { a = b; return; }
  const double n = (double)(a.n + b.n);
  const double delta = b.mean - a.mean;
  a.mean = a.mean + delta * ((double)b.n / n);
  a.var = a.var + b.var + delta * delta * ((double)a.n * (double)b.n / n);
  a.n += b.n;
}
DEVI double wf_result(const Welford& w) {
  if (w.n <= 1) return 0.0;
  return sqrt(w.var / (double)w.n);
}

}  // namespace tsdb
