// k_reduce.hip — SGIterator value computation (SpanGroup.java:632-784) and the
// Aggregators over spans (Aggregators.java:76-243), per emission time t in G.
//
// Closed form (checked against the oracle):
//   non-rate: span s active at t iff first_s <= t <= L_s; cur = last point
//     <= t, nxt = cur+1; value = y_cur if x_cur == t else lerp(cur, nxt, t),
//     int lerp y0 + (t-x0)*(y1-y0)/(x1-x0) in wrapping long with truncating
//     division, double lerp y0 + ((double)(t-x0)*(y1-y0))/(double)(x1-x0).
//     isFloat(t) = OR over spans of [active & float(cur)] | [float(nxt)].
//   rate: active iff |E_s| >= 2 and t <= L_s; cur = last point j>=1 with
//     ts <= t else e_0 (quirk Q5); value = (y_cur - y_prev)/(x_cur - x_prev)
//     with prev = (0,0) for e_0. Always the double path.
//
// Work unit: one wave = 64 consecutive grid indices (a tile, lane = t) x a
// chunk of spans processed in span order, so every lane accumulates exactly
// in the reference's order inside its chunk. Each span's points are placed
// on the tile with O(1) grid ranks: the points falling inside the tile give a
// 64-bit mask M, and lane l's bracket is cur = j + popc(M & le(l)) - 1.
// Chunks are combined in chunk order by k_finalize_* (exact for integers;
// double sums / dev within 1e-9 unless TSDBHIP_EXACT_ORDER forces 1 chunk).
#pragma once
#include "dev_common.h"
#include "k_grid.hip"

namespace tsdb {

enum { MODE_INT = 0, MODE_DBL = 1, MODE_DUAL = 2 };

struct FinalArgs {
  uint64_t T;
  uint32_t n_chunks;
  const uint32_t* grid;
  uint64_t fstar;            // max float-first ts + 1 (0: none)
  int32_t rate;
  int64_t* out_ts;
  uint8_t* out_isint;
  int64_t* out_bits;
  unsigned long long* nan_t; // [1] min t index with NaN/Inf double
  uint64_t g_base;           // global index of point 0 (a rank's slice of G; nan_t is global)
  uint64_t stride;           // partials' stride between chunks (0: T)
};

struct ReduceArgs {
  const uint64_t* e_off;
  const uint32_t* e_len;
  const uint32_t* e_ts;
  const int64_t* e_val;
  const uint8_t* e_flt;
  uint32_t n_kept;
  const uint32_t* grid;
  uint64_t T;
  const uint32_t* bitmap;
  const uint32_t* word_rank;
  int64_t lo;
  uint32_t spans_per_chunk;
  uint32_t n_chunks;
  uint32_t tiles_per_wave;
  uint32_t n_tile_groups;
  uint32_t* ptr;        // [n_waves * spans_per_chunk] per-wave span cursors j
  // per-wave span bracket cache (same indexing as ptr): after a tile, for
  // cursor j (first point past the tile): x/y/type of points j-1 and j (rate:
  // the rate value of point j-1), so a span without points in the next tile
  // is evaluated from registers
  uint2* st_x;          // (x_{j-1}, x_j)    x_j = UINT32_MAX past the end
  longlong2* st_y;      // (y_{j-1}, y_j)
  double* st_rv;        // rate value at point j-1
  uint32_t* st_f;       // bit0 float(j-1), bit1 float(j), bit2 cache valid
  // partials [n_chunks][T]
  uint32_t* p_cnt;
  uint8_t* p_flag;      // bit0 isFloat contribution, bit1 first double is NaN
  int64_t* p_i;
  double* p_d;
  double* p_wim;
  double* p_wiv;
  double* p_wdm;
  double* p_wdv;
  uint32_t* p_dhas;     // double min/max: a non-NaN value was seen
  // initial per-t state ([T] slot layout, null: none): the reduction
  // continues from it (the sequential pass over the ranks of a sharded
  // group: rank r starts from rank r-1's state, so values are pushed in span
  // order across ranks)
  const uint32_t* i_cnt;
  const uint8_t* i_flag;
  const int64_t* i_i;
  const double* i_d;
  const uint32_t* i_dhas;
  const double* i_wim;
  const double* i_wiv;
  const double* i_wdm;
  const double* i_wdv;
  const uint32_t* chunk_e;  // [n_chunks] chunk holds an E (non-direct) span
  uint64_t fstar;           // F* (FinalArgs.fstar): t + 1 < F* is a double t
  int32_t exact;            // TSDBHIP_EXACT_ORDER: IEEE division in the double lerp
  // direct spans (k_direct.hip; d_info null: none): values read from the
  // reference's value bytes at grid rank - d_ga
  const uint32_t* d_info;
  const uint32_t* d_n;
  const uint32_t* d_ga;
  const uint64_t* d_voff;
  const uint32_t* d_x0;
  const uint32_t* d_step;
  const uint32_t* d_c0;
  const uint64_t* d_r0;
  const uint64_t* span_row_start;
  const uint32_t* kept;
  const uint32_t* row_cpre;
  const uint32_t* row_ncells;
  const uint64_t* row_val_off;
  const uint8_t* val;
  // the span state above (cursors, bracket caches, E offsets / lengths) kept
  // in each wave's LDS (dynamic, red_lds_stride bytes a wave) instead of the
  // global st_* arrays: a long grid re-reads it every tile
  uint32_t lds_state;
  // in-kernel finalize (k_reduce only; null: the finalize kernels run after):
  // the last of a tile group's n_chunks waves to finish (tg_done[tg] counts
  // them, and is reset to 0 by that wave) merges the chunks in order and
  // finalizes the group's points into `fin` (the caller's mapped result
  // buffers: the results cross PCIe while the other waves still compute)
  uint32_t* tg_done;
  FinalArgs fin;
};

// LDS bytes of one span's state (y pair, x pair, E offset, [rate value],
// cursor, flags, E length); a wave's region, 16-byte aligned
__host__ __device__ constexpr uint32_t red_lds_span_bytes(bool rate) { return rate ? 52u : 44u; }
__host__ __device__ inline uint64_t red_lds_stride(uint32_t spc, bool rate) { return ((uint64_t)spc * red_lds_span_bytes(rate) + 15) & ~15ull; }

// value bits of a direct span's cell (width 8: long / double bits; width 4:
// int or float widened to double, RowSeq.java:194-226)
DEVI int64_t direct_bits(uint64_t raw, uint32_t info) {
  if (info & 4u /*DIR_W8*/) return (int64_t)bswap64(raw);
  const uint32_t u = bswap32((uint32_t)raw);
  if (info & 2u /*DIR_FLT*/) return dbits((double)__uint_as_float(u));
  return (int64_t)(int32_t)u;
}
DEVI uint64_t direct_load(const uint8_t* p, uint32_t info) {
  return (info & 4u) ? *(const uint64_t*)p : (uint64_t)*(const uint32_t*)p;
}

// byte offset of E index e of a direct span whose points cross rows
DEVI uint64_t direct_multi_off(const ReduceArgs& r, uint32_t k, int64_t e) {
  const uint32_t s = r.kept[k];
  const uint64_t r0 = r.span_row_start[s], r1 = r.span_row_start[s + 1];
  const uint32_t c = r.d_c0[k] + (uint32_t)e;
  uint64_t lo = r0, hi = r1 - 1;  // last row with cpre <= c
  while (lo < hi) {
    const uint64_t mid = (lo + hi + 1) >> 1;
    if (r.row_cpre[mid] <= c) lo = mid; else hi = mid - 1;
  }
  const uint32_t w = (r.d_info[k] & 4u) ? 8u : 4u;
  return r.row_val_off[lo] + (uint64_t)w * (c - r.row_cpre[lo]);
}

struct Acc {
  uint32_t cnt;
  uint32_t flag;   // bit0 float contribution, bit1 first double value is NaN
  uint32_t dhas;
  int64_t ia;
  double da;
  Welford wi, wd;
  bool fastdiv;    // wd pushes through wf_push_rcp (not EXACT_ORDER)
};

DEVI void acc_init(Acc& a) {
  a.cnt = 0; a.flag = 0; a.dhas = 0; a.ia = 0; a.da = 0;
  wf_init(a.wi); wf_init(a.wd);
  a.fastdiv = false;
}

template <int AGG, int MODE>
DEVI void acc_push(Acc& a, int64_t yi, double yd) {
  const bool first = a.cnt == 0;
  if (MODE != MODE_DBL) {
    if (AGG == 4) wf_push(a.wi, (double)yi);
    else if (first) a.ia = yi;
    else if (AGG == 1) { if (yi < a.ia) a.ia = yi; }
    else if (AGG == 2) { if (yi > a.ia) a.ia = yi; }
    else a.ia = ladd(a.ia, yi);
  }
  if (MODE != MODE_INT) {
    if (AGG == 4) {
      if (a.fastdiv) wf_push_rcp(a.wd, yd);
      else wf_push(a.wd, yd);
    }
    else if (AGG == 1 || AGG == 2) {
      if (yd != yd) { if (first) a.flag |= 2u; }
      else if (!a.dhas) { a.da = yd; a.dhas = 1; }
      else if (AGG == 1 ? (yd < a.da) : (yd > a.da)) a.da = yd;
    } else {
      a.da = first ? yd : a.da + yd;
    }
  }
  a.cnt++;
}

// A precedes B in span order.
template <int AGG, int MODE>
DEVI void acc_merge(Acc& a, const Acc& b) {
  if (b.cnt == 0) { a.flag |= (b.flag & 1u); return; }
  if (a.cnt == 0) { const uint32_t f = a.flag & 1u; a = b; a.flag |= f; return; }
  if (MODE != MODE_DBL) {
    if (AGG == 4) wf_merge(a.wi, b.wi);
    else if (AGG == 1) { if (b.ia < a.ia) a.ia = b.ia; }
    else if (AGG == 2) { if (b.ia > a.ia) a.ia = b.ia; }
    else a.ia = ladd(a.ia, b.ia);
  }
  if (MODE != MODE_INT) {
    if (AGG == 4) wf_merge(a.wd, b.wd);
    else if (AGG == 1 || AGG == 2) {
      if (!a.dhas) { a.da = b.da; a.dhas = b.dhas; }
      else if (b.dhas && (AGG == 1 ? (b.da < a.da) : (b.da > a.da))) a.da = b.da;
    } else {
      a.da = a.da + b.da;
    }
  }
  a.flag |= (b.flag & 1u);  // first-NaN bit stays A's
  a.cnt += b.cnt;
}

template <int AGG, int MODE>
DEVI void acc_store(const ReduceArgs& r, uint64_t p, const Acc& a) {
  r.p_cnt[p] = a.cnt;
  if (MODE == MODE_DUAL || AGG == 1 || AGG == 2) r.p_flag[p] = (uint8_t)a.flag;
  if (MODE != MODE_DBL && AGG != 4) r.p_i[p] = a.ia;
  if (MODE != MODE_INT && AGG != 4) r.p_d[p] = a.da;
  if (MODE != MODE_INT && (AGG == 1 || AGG == 2)) r.p_dhas[p] = a.dhas;
  if (AGG == 4) {
    if (MODE != MODE_DBL) { r.p_wim[p] = a.wi.mean; r.p_wiv[p] = a.wi.var; }
    if (MODE != MODE_INT) { r.p_wdm[p] = a.wd.mean; r.p_wdv[p] = a.wd.var; }
  }
}

// the initial state of t (ReduceArgs.i_*), or empty
template <int AGG, int MODE>
DEVI void acc_start(const ReduceArgs& r, uint64_t g, Acc& a) {
  acc_init(a);
  if (!r.i_cnt) return;
  a.cnt = r.i_cnt[g];
  if (MODE == MODE_DUAL || AGG == 1 || AGG == 2) a.flag = r.i_flag[g];
  if (MODE != MODE_DBL && AGG != 4) a.ia = r.i_i[g];
  if (MODE != MODE_INT && AGG != 4) a.da = r.i_d[g];
  if (MODE != MODE_INT && (AGG == 1 || AGG == 2)) a.dhas = r.i_dhas[g];
  if (AGG == 4) {
    if (MODE != MODE_DBL) { a.wi.n = a.cnt; a.wi.mean = r.i_wim[g]; a.wi.var = r.i_wiv[g]; }
    if (MODE != MODE_INT) { a.wd.n = a.cnt; a.wd.mean = r.i_wdm[g]; a.wd.var = r.i_wdv[g]; }
  }
}

template <int AGG, int MODE>
DEVI void acc_load(const ReduceArgs& r, uint64_t p, Acc& a) {
  acc_init(a);
  a.cnt = r.p_cnt[p];
  if (MODE == MODE_DUAL || AGG == 1 || AGG == 2) a.flag = r.p_flag[p];
  if (MODE != MODE_DBL && AGG != 4) a.ia = r.p_i[p];
  if (MODE != MODE_INT && AGG != 4) a.da = r.p_d[p];
  if (MODE != MODE_INT && (AGG == 1 || AGG == 2)) a.dhas = r.p_dhas[p];
  if (AGG == 4) {
    if (MODE != MODE_DBL) { a.wi.n = a.cnt; a.wi.mean = r.p_wim[p]; a.wi.var = r.p_wiv[p]; }
    if (MODE != MODE_INT) { a.wd.n = a.cnt; a.wd.mean = r.p_wdm[p]; a.wd.var = r.p_wdv[p]; }
  }
}


template <int AGG, int MODE, bool RATE>
DEVI void finalize_one(const FinalArgs& f, uint64_t g, const Acc& a) {
  const int64_t t = f.grid[g];
  const bool isflt = RATE || MODE == MODE_DBL || (a.flag & 1u) || ((uint64_t)t + 1 < f.fstar);
  int64_t bits;
  if (isflt) {
    double d;
    if (AGG == 0) d = a.da;
    else if (AGG == 3) d = a.da / (double)(int32_t)a.cnt;
    else if (AGG == 4) d = wf_result(a.wd);
    else d = (a.flag & 2u) ? __longlong_as_double(0x7ff8000000000000LL) : a.da;
    if (d != d || isinf(d)) atomicMin(f.nan_t, (unsigned long long)(f.g_base + g));
    bits = dbits(d);
  } else {
    if (AGG == 3) bits = ldiv(a.ia, (int64_t)(int32_t)a.cnt);
    // (integer dev: the caller reduces in one span-ordered pass, so this is
    // the reference's sequential Welford, :196-217)
    else if (AGG == 4) bits = d2l(wf_result(a.wi));
    else bits = a.ia;
  }
  f.out_ts[g] = t;
  f.out_isint[g] = isflt ? 0 : 1;
  f.out_bits[g] = bits;
}

// Java long lerp: y0 + (x - x0) * (y1 - y0) / (x1 - x0), 0 < x1 - x0 < 2^32.
DEVI int64_t lerp_long(int64_t x, int64_t x0, int64_t y0, int64_t x1, int64_t y1) {
  const int64_t num = lmul(x - x0, lsub(y1, y0));
  const uint32_t d = (uint32_t)(x1 - x0);  // timestamps are u32: 0 < d < 2^32
  const uint64_t mag = num < 0 ? (uint64_t)0 - (uint64_t)num : (uint64_t)num;
  const uint64_t q = udiv64_32(mag, d);
  const int64_t sq = num < 0 ? (int64_t)((uint64_t)0 - q) : (int64_t)q;
  return ladd(y0, sq);
}
DEVI double lerp_double(int64_t x, int64_t x0, double y0, int64_t x1, double y1) {
  return y0 + ((double)(x - x0) * (y1 - y0)) / (double)(x1 - x0);
}
// The long lerp of a bracket fixed over a tile, prepared once per span
// (lane-parallel): im = |y1 - y0| with bit 31 its sign, or UINT32_MAX when
// |y1 - y0| >= 2^31 - 1; magr = |y1 - y0| / (x1 - x0).
DEVI void lerp_long_prep(int64_t y0, int64_t y1, uint32_t d, uint32_t& im, double& magr) {
  const int64_t dy = lsub(y1, y0);
  const uint64_t mag = dy < 0 ? (uint64_t)0 - (uint64_t)dy : (uint64_t)dy;
  im = UINT32_MAX;
  magr = 0.0;
  if (mag < 0x7fffffffull && d > 0) {
    im = (uint32_t)mag | (dy < 0 ? 0x80000000u : 0u);
    magr = (double)mag / (double)d;
  }
}
// lerp_long for 0 < u = x - x0 < d = x1 - x0 and a prepared im != UINT32_MAX:
// the product u * dy cannot wrap, and its truncated quotient by d is the
// double estimate u * magr (error < 2^-20) made exact by one remainder check.
DEVI int64_t lerp_long_prepped(uint32_t u, uint32_t d, int64_t y0, uint32_t im, double magr) {
  const uint32_t mag = im & 0x7fffffffu;
  uint32_t q = (uint32_t)((double)u * magr);
  const int64_t rem = (int64_t)((uint64_t)u * mag) - (int64_t)((uint64_t)q * d);
  q = rem < 0 ? q - 1u : (rem >= (int64_t)d ? q + 1u : q);
  return ladd(y0, (im >> 31) ? -(int64_t)q : (int64_t)q);
}

// acc_push on active lanes only, without a branch: the push is computed on
// a copy and selected (no exec-mask juggling on the scalar unit).
template <int AGG, int MODE>
DEVI void acc_push_if(Acc& a, bool act, int64_t yi, double yd) {
  Acc b = a;
  acc_push<AGG, MODE>(b, yi, yd);
  a.cnt = act ? b.cnt : a.cnt;
  a.flag = act ? b.flag : a.flag;
  a.dhas = act ? b.dhas : a.dhas;
  a.ia = act ? b.ia : a.ia;
  a.da = act ? b.da : a.da;
  a.wi.n = act ? b.wi.n : a.wi.n;
  a.wi.mean = act ? b.wi.mean : a.wi.mean;
  a.wi.var = act ? b.wi.var : a.wi.var;
  a.wd.n = act ? b.wd.n : a.wd.n;
  a.wd.mean = act ? b.wd.mean : a.wd.mean;
  a.wd.var = act ? b.wd.var : a.wd.var;
}

template <uint32_t W, bool FLT>
DEVI int64_t dbits_of(uint64_t raw) {
  if (W == 8) return (int64_t)bswap64(raw);
  const uint32_t u = bswap32((uint32_t)raw);
  if (FLT) return dbits((double)__uint_as_float(u));
  return (int64_t)(int32_t)u;
}
template <uint32_t W>
DEVI uint64_t dload(const uint8_t* p) {
  if (W == 8) return *(const uint64_t*)p;
  return (uint64_t)*(const uint32_t*)p;
}

// A run of `run` (<= 8) single-row direct spans of one value width and type,
// batch lanes i..i+run-1: all value loads issued first, branch-free
// (inactive lanes read E[0]), then pushed in span order.
template <int AGG, int MODE, bool RATE, uint32_t W, bool FLT>
DEVI void direct_run(const ReduceArgs& r, Acc& acc, uint32_t run, uint32_t i, uint64_t dvo_l, uint32_t dga_l,
                     uint32_t dn_l, uint32_t dx0_l, uint32_t dstep_l, uint64_t g, bool gv) {
  uint64_t raw[8], rawp0[8];
  bool act[8];
  int64_t ev[8];
#pragma unroll
  for (uint32_t u = 0; u < 8; u++) {
    // (past the run: repeat its last span, so the loads stay straight-line)
    const int ln = (int)(i + min(u, run - 1));
    const uint32_t ga = readlane_u32(dga_l, ln), n = readlane_u32(dn_l, ln);
    const uint64_t vo = readlane_u64(dvo_l, ln);
    const int64_t e = (int64_t)g - (int64_t)ga;
    ev[u] = e;
    act[u] = gv && (RATE ? (n >= 2 && e <= (int64_t)n - 2) : (e >= 0 && e < (int64_t)n));
    const int64_t ec = act[u] ? (RATE ? (e < 0 ? 0 : e + 1) : e) : 0;
    raw[u] = dload<W>(r.val + vo + W * (uint64_t)ec);
    if (RATE) {  // lane 0's previous cell (the other lanes take their neighbour's)
      const int64_t ep = (lane_id() == 0 && act[u] && e >= 0) ? e : ec;
      rawp0[u] = dload<W>(r.val + vo + W * (uint64_t)ep);
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // keep every load of the run ahead of the first use
#pragma unroll
  for (uint32_t u = 0; u < 8; u++) {
    if (u >= run) break;
    const int64_t b = dbits_of<W, FLT>(raw[u]);
    if (RATE) {
      const uint32_t step = readlane_u32(dstep_l, (int)(i + u));
      const double diff = to_double(b, FLT) - to_double(dbits_of<W, FLT>(wave_shr1_u64(raw[u], rawp0[u])), FLT);
      double v;
      // x_cur - x_prev = step; a power-of-two step divides exactly as a
      // product with its (exact) reciprocal: same IEEE result, no divide
      if ((step & (step - 1)) == 0) v = diff * __builtin_amdgcn_ldexp(1.0, -(int)__builtin_ctz(step));
      else v = diff / (double)(int64_t)step;
      if (ballot(act[u] && ev[u] < 0)) {  // Q5: before the span's second point, y0 / x0
        const uint32_t x0 = readlane_u32(dx0_l, (int)(i + u));
        if (ev[u] < 0) v = to_double(b, FLT) / (double)(int64_t)x0;
      }
      acc_push_if<AGG, MODE>(acc, act[u], 0, v);
    } else {
      if (MODE == MODE_DUAL && FLT && act[u]) acc.flag |= 1u;
      acc_push_if<AGG, MODE>(acc, act[u], b, MODE == MODE_INT ? 0.0 : to_double(b, MODE == MODE_DBL || FLT));
    }
  }
}

// DONLY: the instantiation for span chunks holding direct spans only (no E
// span state, fewer registers); with direct spans present both are launched
// and each takes the chunks r.chunk_e marks as its own.
// reduce_wave: the work of one wave (tile group x span chunk) of a group;
// k_reduce runs one group, k_reduce_seg (k_group.hip) many groups per launch.
template <int AGG, int MODE, bool RATE, bool DONLY>
DEVI void reduce_wave_body(const ReduceArgs& r, const uint32_t wave, uint8_t* lds_w, const uint32_t chunk,
                           const uint32_t tg);
template <int AGG, int MODE, bool RATE, bool DONLY>
DEVI void reduce_wave(const ReduceArgs& r, const uint32_t wave, uint8_t* lds_w) {
  const uint32_t n_waves = r.n_chunks * r.n_tile_groups;
  if (wave >= n_waves) return;
  const uint32_t chunk = wave % r.n_chunks;
  const uint32_t tg = wave / r.n_chunks;
  // (no chunk flags: the general instantiation takes every chunk)
  if (r.d_info && r.chunk_e && (r.chunk_e[chunk] != 0) == DONLY) return;  // the other instantiation's chunk
  if ((!r.d_info || !r.chunk_e) && DONLY) return;
  reduce_wave_body<AGG, MODE, RATE, DONLY>(r, wave, lds_w, chunk, tg);
  if (!r.tg_done) return;
  // this chunk's partials of tile group tg are stored: release them; the
  // group's last wave acquires every chunk's and finalizes the group
  const int lane = lane_id();
  __threadfence();
  uint32_t prev = 0;
  if (lane == 0) prev = atomicAdd(&r.tg_done[tg], 1u);
  prev = __builtin_amdgcn_readfirstlane(prev);
  if (prev != r.n_chunks - 1) return;
  __threadfence();
  if (lane == 0) r.tg_done[tg] = 0u;  // (zero for the next call)
  const uint64_t n_tiles = (r.T + WAVE - 1) / WAVE;
  const uint64_t tb = (uint64_t)tg * r.tiles_per_wave, te = min(n_tiles, tb + r.tiles_per_wave);
  for (uint64_t t = tb; t < te; t++) {
    const uint64_t g = t * WAVE + lane;
    if (g >= r.T) break;
    Acc a;
    acc_load<AGG, MODE>(r, g, a);
    for (uint32_t c = 1; c < r.n_chunks; c++) {
      Acc b;
      acc_load<AGG, MODE>(r, (uint64_t)c * r.T + g, b);
      acc_merge<AGG, MODE>(a, b);
    }
    finalize_one<AGG, MODE, RATE>(r.fin, g, a);
  }
}

template <int AGG, int MODE, bool RATE, bool DONLY>
DEVI void reduce_wave_body(const ReduceArgs& r, const uint32_t wave, uint8_t* lds_w, const uint32_t chunk,
                           const uint32_t tg) {
  const int lane = lane_id();
  const uint32_t k0 = chunk * r.spans_per_chunk;
  const uint32_t k1 = min(r.n_kept, k0 + r.spans_per_chunk);
  const uint64_t n_tiles = (r.T + WAVE - 1) / WAVE;
  const uint64_t tb = (uint64_t)tg * r.tiles_per_wave;
  const uint64_t te = min(n_tiles, tb + r.tiles_per_wave);
  if (tb >= te || k0 >= k1) {
    // still write empty partials for this chunk's tiles
    for (uint64_t t = tb; t < te; t++) {
      const uint64_t g = t * WAVE + lane;
      if (g < r.T) { Acc a; acc_start<AGG, MODE>(r, g, a); acc_store<AGG, MODE>(r, (uint64_t)chunk * r.T + g, a); }
    }
    return;
  }
  // span state, indexed by k - k0: this wave's LDS region, or global
  const uint32_t spc = r.spans_per_chunk;
  const uint64_t so = (uint64_t)wave * spc;
  uint32_t* ptr = r.ptr + so;
  uint32_t* S_f = r.st_f + so;
  uint2* S_x = r.st_x + so;
  longlong2* S_y = r.st_y + so;
  double* S_rv = r.st_rv + so;
  const uint64_t* S_eo = r.e_off + k0;
  const uint32_t* S_len = r.e_len + k0;
  uint64_t* L_eo = nullptr;
  uint32_t* L_len = nullptr;
  if (lds_w) {
    S_y = (longlong2*)lds_w;
    S_x = (uint2*)(S_y + spc);
    L_eo = (uint64_t*)(S_x + spc);
    S_rv = (double*)(L_eo + spc);
    ptr = (uint32_t*)(RATE ? (uint8_t*)(S_rv + spc) : (uint8_t*)S_rv);
    S_f = ptr + spc;
    L_len = S_f + spc;
    S_eo = L_eo;
    S_len = L_len;
  }
  const uint32_t base_idx = RATE ? 1u : 0u;
  // cursor init: first point index >= base_idx with ts >= G[tb*64]
  if (!DONLY) {
    const int64_t t0 = r.grid[tb * WAVE];
    for (uint32_t k = k0 + lane; k < k1; k += WAVE) {
      const uint32_t sl = k - k0;
      if (r.d_info && (r.d_info[k] & 1u)) { ptr[sl] = 0; S_f[sl] = 0; continue; }
      const uint64_t eo = r.e_off[k];
      const uint32_t len = r.e_len[k];
      if (L_eo) { L_eo[sl] = eo; L_len[sl] = len; }
      uint32_t lo = base_idx, hi = len;
      if (hi < lo) hi = lo;
      // a span that starts at/after the wave's first grid point (every span
      // of a single-tile grid: C3*) has its cursor at base_idx: one load
      // instead of a dependent binary search
      if (lo < hi && (int64_t)r.e_ts[eo + lo] >= t0) hi = lo;
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((int64_t)r.e_ts[eo + mid] < t0) lo = mid + 1; else hi = mid;
      }
      ptr[k - k0] = lo;
      // the bracket cache for cursor lo (points lo-1 and lo), filled here
      // lane-parallel so the first tile needs no per-span loads
      const uint32_t j = lo;
      uint2 x = make_uint2(0, UINT32_MAX);
      longlong2 y = make_longlong2(0, 0);
      uint32_t f = 4u;
      double rv = 0.0;
      if (j >= 1 && j <= len) {
        x.x = r.e_ts[eo + j - 1];
        y.x = r.e_val[eo + j - 1];
        if (r.e_flt[eo + j - 1]) f |= 1u;
      }
      if (j < len) {
        x.y = r.e_ts[eo + j];
        y.y = r.e_val[eo + j];
        if (r.e_flt[eo + j]) f |= 2u;
      }
      if (RATE && j >= 1 && j <= len) {
        const double yc = to_double(y.x, (f & 1u) != 0);
        if (j >= 2) {
          const int64_t xp = r.e_ts[eo + j - 2];
          const double yp = to_double(r.e_val[eo + j - 2], r.e_flt[eo + j - 2] != 0);
          rv = (yc - yp) / (double)((int64_t)x.x - xp);
        } else {
          rv = yc / (double)(int64_t)x.x;  // Q5: prev = (0, 0)
        }
      }
      S_x[sl] = x;
      S_y[sl] = y;
      if (RATE) S_rv[sl] = rv;
      S_f[sl] = f;
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");

  for (uint64_t tile = tb; tile < te; tile++) {
    const uint64_t g0 = tile * WAVE;
    const uint64_t g = g0 + lane;
    const bool gv = g < r.T;
    const int nvalid = (int)min((uint64_t)WAVE, r.T - g0);
    const uint64_t vmask = nvalid == 64 ? ~0ull : ((1ull << nvalid) - 1);
    const int64_t tl = gv ? (int64_t)r.grid[g] : INT64_MAX;
    const int64_t t_first = (int64_t)r.grid[g0];
    const int64_t t_last = (int64_t)r.grid[g0 + nvalid - 1];
    Acc acc;
    if (gv) acc_start<AGG, MODE>(r, g, acc);
    else acc_init(acc);
    acc.fastdiv = AGG == 4 && MODE != MODE_INT && !r.exact;
    // dual mode: t before the latest float-first point is on the double path
    // whatever the spans hold (F*, SpanGroup.java:632-645); once every lane's
    // t is known to be double, no long lerp of this tile is ever read
    if (MODE == MODE_DUAL && gv && (uint64_t)tl + 1 < r.fstar) acc.flag |= 1u;
    auto need_long = [&](bool fa, bool fb) {
      if (MODE == MODE_INT) return true;
      if (MODE != MODE_DUAL || fa || fb) return false;
      return ballot(gv && !(acc.flag & 1u)) != 0;
    };
    // Spans in order, 64 at a time: their E offsets/lengths come in with one
    // load per lane. A span whose E holds exactly this tile's grid points
    // (E[g0 .. g0+n) == G[g0 .. g0+n): aligned series) needs no bracket
    // search and no lerp: lane l takes E[g0 + l]; runs of such spans load
    // their values up to 8 spans ahead. Every other span takes the general
    // path (cursor, grid ranks, lerp / rate).
    auto general = [&](uint32_t k, uint64_t eo, uint32_t len, uint32_t j) -> uint32_t {
      const int64_t first = r.e_ts[eo], last = r.e_ts[eo + len - 1];
      if (RATE) {
        if (len < 2 || last < t_first) return j;
      } else {
        if (first > t_last || last < t_first) return j;  // not started (F*) / expired
      }
      const uint32_t idx = j + lane;
      const int64_t pts = idx < len ? (int64_t)r.e_ts[eo + idx] : INT64_MAX;
      const bool in = pts <= t_last;
      const uint64_t inmask = ballot(in);
      const int kk = __popcll(inmask);
      uint64_t M;
      if (kk == nvalid) {
        M = vmask;  // every grid point of the tile is a point of this span
      } else if (kk) {
        uint64_t bit = 0;
        if (in) bit = 1ull << (grid_rank(r.bitmap, r.word_rank, r.lo, pts) - g0);
        M = wave_or_u64(bit);
      } else {
        M = 0;
      }
      const uint32_t jn = j + kk;
      const int cl = __popcll(M & lanemask_le(lane));
      const int64_t cur = (int64_t)j + cl - 1;
      // bracket timestamps: inside the tile they are this wave's loaded points
      const int64_t ts_in = (int64_t)shfl_u64((uint64_t)pts, cl > 0 ? cl - 1 : 0);
      if (!gv) return jn;
      if (RATE) {
        if (tl > last) return jn;
        const int64_t xc = cl > 0 ? ts_in : (int64_t)r.e_ts[eo + cur];
        const double yc = to_double(r.e_val[eo + cur], r.e_flt[eo + cur] != 0);
        double yp = 0.0;
        int64_t xp = 0;
        if (cur >= 1) { xp = r.e_ts[eo + cur - 1]; yp = to_double(r.e_val[eo + cur - 1], r.e_flt[eo + cur - 1] != 0); }
        acc_push<AGG, MODE>(acc, 0, (yc - yp) / (double)(xc - xp));
        return jn;
      }
      if (cur < 0) {  // not started: next slot holds e_0
        if (MODE == MODE_DUAL && r.e_flt[eo]) acc.flag |= 1u;
        return jn;
      }
      const int64_t xc = cl > 0 ? ts_in : (int64_t)r.e_ts[eo + cur];
      const bool active = (uint32_t)cur < len - 1 || xc == tl;
      if (!active) return jn;  // expired: nothing in either slot
      const int64_t vc = r.e_val[eo + cur];
      bool fc = false, fn = false;
      if (MODE == MODE_DUAL) {
        fc = r.e_flt[eo + cur] != 0;
        if ((uint32_t)cur + 1 < len) fn = r.e_flt[eo + cur + 1] != 0;
        if (fc || fn) acc.flag |= 1u;
      }
      if (xc == tl) {
        acc_push<AGG, MODE>(acc, vc, MODE == MODE_INT ? 0.0 : to_double(vc, MODE == MODE_DBL || fc));
      } else {
        const int64_t xn = r.e_ts[eo + cur + 1];
        const int64_t vn = r.e_val[eo + cur + 1];
        int64_t yi = 0;
        double yd = 0.0;
        // (dual: a float in the bracket puts t on the double path; the long
        // lerp of this span is then never read)
        if (need_long(fc, fn)) yi = lerp_long(tl, xc, vc, xn, vn);
        if (MODE != MODE_INT)
          yd = lerp_double(tl, xc, to_double(vc, MODE == MODE_DBL || fc), xn,
                           to_double(vn, MODE == MODE_DBL || fn));
        acc_push<AGG, MODE>(acc, yi, yd);
      }
      return jn;
    };
    // A direct span (k_direct.hip) at lane g: E index e = g - ga; its value
    // is the cell itself (non-rate: active iff 0 <= e < n), or its constant-
    // step difference (rate: e = j - 1 for point j; e < 0 is the Q5 state
    // cur = e_0, prev = (0, 0); active iff n >= 2 and e <= n - 2).
    auto direct_push = [&](uint32_t info, bool act, int64_t e, uint64_t raw, uint64_t rawp, uint32_t x0,
                           uint32_t step) {
      if (!act) return;
      const bool flt = (info & 2u) != 0;
      const int64_t b = direct_bits(raw, info);
      if (RATE) {
        double v;
        if (e < 0) {
          v = to_double(b, flt) / (double)(int64_t)x0;
        } else {
          const double diff = to_double(b, flt) - to_double(direct_bits(rawp, info), flt);
          // x_cur - x_prev = step; a power-of-two step divides exactly as a
          // product with its (exact) reciprocal: same IEEE result, no divide
          if ((step & (step - 1)) == 0) v = diff * __builtin_amdgcn_ldexp(1.0, -(int)__builtin_ctz(step));
          else v = diff / (double)(int64_t)step;
        }
        acc_push<AGG, MODE>(acc, 0, v);
        return;
      }
      if (MODE == MODE_DUAL && flt) acc.flag |= 1u;
      acc_push<AGG, MODE>(acc, b, MODE == MODE_INT ? 0.0 : to_double(b, MODE == MODE_DBL || flt));
    };
    // one direct span, any row layout
    auto direct_one = [&](uint32_t k, uint32_t info, uint32_t ga, uint32_t n, uint64_t vo) {
      const int64_t e = (int64_t)g - (int64_t)ga;
      const bool act = gv && (RATE ? (n >= 2 && e <= (int64_t)n - 2) : (e >= 0 && e < (int64_t)n));
      const int64_t ec = RATE ? (e < 0 ? 0 : e + 1) : e;  // the cell read
      const bool multi = (info & 8u) != 0;
      uint64_t raw = 0, rawp = 0;
      if (act) raw = direct_load(r.val + (multi ? direct_multi_off(r, k, ec) : vo + ((info & 4u) ? 8 : 4) * ec), info);
      uint32_t x0 = 0, step = 0;
      if (RATE) {
        rawp = shfl_up_u64(raw, 1);
        if (lane == 0 && act && e >= 0)
          rawp = direct_load(r.val + (multi ? direct_multi_off(r, k, e) : vo + ((info & 4u) ? 8 : 4) * e), info);
        x0 = r.d_x0[k];
        step = r.d_step[k];
      }
      direct_push(info, act, e, raw, rawp, x0, step);
    };
    constexpr bool ALIGNED_OK = !RATE && MODE != MODE_DUAL;
    constexpr bool LIN_OK = !RATE && MODE != MODE_INT && (AGG == 0 || AGG == 3);
    for (uint32_t kb = k0; kb < k1; kb += WAVE) {
      const uint32_t kl = kb + lane;
      const bool kv = kl < k1;
      const uint32_t dinfo_l = (r.d_info && kv) ? r.d_info[kl] : 0u;
      const bool dl = DONLY || (dinfo_l & 1u) != 0;
      const uint32_t sl = kl - k0;
      const uint64_t eo_l = kv && !dl ? S_eo[sl] : 0;
      const uint32_t len_l = kv && !dl ? S_len[sl] : 0;
      // E spans: cursor and bracket cache, lane = span
      const bool el = !DONLY && kv && !dl;
      uint32_t j_l = 0, f_l = 0;
      uint2 x_l = make_uint2(0, 0);
      longlong2 y_l = make_longlong2(0, 0);
      double rv_l = 0.0;
      if (el) {
        j_l = ptr[sl];
        f_l = S_f[sl];
        if (f_l & 4u) {
          x_l = S_x[sl];
          y_l = S_y[sl];
          if (RATE) rv_l = S_rv[sl];
        }
      }
      bool dirty_l = false;
      // per-span doubles of the cached bracket (lane = span): y0, y1 - y0,
      // 1 / (x1 - x0)
      double y0d_l = 0.0, dyd_l = 0.0, rinv_l = 0.0;
      if (!RATE && MODE != MODE_INT && el && (f_l & 4u) && x_l.y > x_l.x) {
        y0d_l = to_double(y_l.x, MODE == MODE_DBL || (f_l & 1u));
        dyd_l = to_double(y_l.y, MODE == MODE_DBL || (f_l & 2u)) - y0d_l;
        rinv_l = 1.0 / (double)(x_l.y - x_l.x);
      }
      // the long lerp of the cached bracket: |y1 - y0| (bit 31: negative), or
      // UINT32_MAX when it is 2^31 - 1 or more (general lerp); |y1 - y0| / d
      uint32_t im_l = UINT32_MAX;
      double magr_l = 0.0;
      // dual mode, every lane's t already on the double path: no long lerp of
      // this batch is read (flags are only ever set), so none is prepared
      const bool dual_all_dbl = MODE == MODE_DUAL && ballot(gv && !(acc.flag & 1u)) == 0;
      if (!RATE && MODE != MODE_DBL && !dual_all_dbl && el && (f_l & 4u) && x_l.y > x_l.x)
        lerp_long_prep(y_l.x, y_l.y, x_l.y - x_l.x, im_l, magr_l);
      const uint64_t dmask = ballot(dl);
      uint32_t dga_l = 0, dn_l = 0, dx0_l = 0, dstep_l = 0;
      uint64_t dvo_l = 0;
      uint64_t dsingle = 0;  // direct spans held in one row
      if (dmask) {
        if (dl) {
          dga_l = r.d_ga[kl]; dn_l = r.d_n[kl]; dvo_l = r.d_voff[kl];
          if (RATE) { dx0_l = r.d_x0[kl]; dstep_l = r.d_step[kl]; }
        }
        dsingle = ballot(dl && !(dinfo_l & 8u));
      }
      uint64_t almask = 0;
      if (ALIGNED_OK) {  // (cursor at g0 first: the end check loads only then)
        bool al = el && j_l == g0 && (uint64_t)len_l >= g0 + (uint64_t)nvalid;
        if (al) al = (int64_t)r.e_ts[eo_l + g0] == t_first && (int64_t)r.e_ts[eo_l + g0 + nvalid - 1] == t_last;
        almask = ballot(al);
      }
      // spans with no point in this tile take the cache
      const bool cl_ok = el && !((almask >> lane) & 1) && (f_l & 4u);
      const uint64_t cmask = ballot(cl_ok && (j_l >= len_l || (int64_t)x_l.y > t_last));
      // Sum / avg of doubles (outside TSDBHIP_EXACT_ORDER): the cached spans
      // active over the whole tile add up to one line in t, sum_s v_s(t_first)
      // + (t - t_first) * sum_s slope_s: two wave sums instead of a lerp per
      // span and lane (C4: ~94% of the span-tiles). Dual mode: int spans only
      // once every lane's t is on the double path (their long lerps are then
      // never read). Non-finite brackets keep the per-span path.
      uint64_t lmask = 0;
      if (LIN_OK && !r.exact) {
        const bool all_dbl = MODE != MODE_DUAL || dual_all_dbl;
        const double sl = dyd_l * rinv_l;
        const double v0 = y0d_l + ((double)(uint32_t)(t_first - (int64_t)x_l.x) * dyd_l) * rinv_l;
        const bool lin = ((cmask >> lane) & 1) && j_l > 0 && j_l < len_l && x_l.y > x_l.x &&
                         (all_dbl || (f_l & 3u)) && __builtin_isfinite(v0) && __builtin_isfinite(sl);
        lmask = ballot(lin);
        if (lmask) {
          double s0 = lin ? v0 : 0.0, s1 = lin ? sl : 0.0;
#pragma unroll
          for (int m = 1; m < WAVE; m <<= 1) {  // (xor butterfly: the same sums in every lane)
            s0 += __longlong_as_double((long long)shfl_xor_u64((uint64_t)__double_as_longlong(s0), m));
            s1 += __longlong_as_double((long long)shfl_xor_u64((uint64_t)__double_as_longlong(s1), m));
          }
          const bool lflt = MODE == MODE_DUAL && ballot(lin && (f_l & 3u)) != 0;
          if (gv) {
            const double y = s0 + (double)(tl - t_first) * s1;
            acc.da = acc.cnt == 0 ? y : acc.da + y;
            acc.cnt += (uint32_t)__popcll(lmask);
            if (lflt) acc.flag |= 1u;
          }
        }
      }
      // spans with exactly one point (j) in this tile: point j+1 loaded here,
      // lane-parallel, so the span needs no load of its own
      uint32_t x2_l = UINT32_MAX, f2_l = 0;
      int64_t y2_l = 0;
      const bool sc = cl_ok && j_l < len_l && (int64_t)x_l.y <= t_last;
      if (sc && j_l + 1 < len_l) {
        x2_l = r.e_ts[eo_l + j_l + 1];
        y2_l = r.e_val[eo_l + j_l + 1];
        f2_l = r.e_flt[eo_l + j_l + 1];
      }
      // (the long lerp of the bracket (j, j+1), prepared as im_l / magr_l)
      uint32_t im2_l = UINT32_MAX;
      double magr2_l = 0.0;
      if (!RATE && MODE != MODE_DBL && !dual_all_dbl && sc && j_l + 1 < len_l && x2_l > x_l.y)
        lerp_long_prep(y_l.y, y2_l, x2_l - x_l.y, im2_l, magr2_l);
      // ... and its double lerp's y0, y1 - y0 and 1 / (x1 - x0) (outside
      // EXACT_ORDER the lanes after point j then lerp as the cached path does:
      // a product with the reciprocal, no division a lane)
      double y0d2_l = 0.0, dyd2_l = 0.0, rinv2_l = 0.0;
      if (!RATE && MODE != MODE_INT && !r.exact && sc && j_l + 1 < len_l && x2_l > x_l.y) {
        y0d2_l = to_double(y_l.y, MODE == MODE_DBL || (f_l & 2u));
        dyd2_l = to_double(y2_l, MODE == MODE_DBL || f2_l != 0) - y0d2_l;
        rinv2_l = 1.0 / (double)(x2_l - x_l.y);
      }
      const uint64_t smask = ballot(sc && (int64_t)x2_l > t_last);
      const uint32_t nb = min((uint32_t)WAVE, k1 - kb);
      // Integer sum / min / max / avg are order-free (wrapping sums, exact
      // min / max), so the cached spans whose long lerp is prepared (C4-int:
      // ~93% of the span-tiles) go first, in a loop of their own: five
      // readlanes, the prepared lerp and the push, instead of the ordered
      // loop's dispatch over six masks and the generic cached(). Sum / avg add
      // the y0s on the scalar unit and the signed quotients per lane.
      constexpr bool INT_FAST = MODE == MODE_INT && !RATE && AGG != 4;
      // cached spans that contribute nothing to this tile (expired; not
      // started, outside rate mode): cached() would return at once, so the
      // ordered loop skips them in runs instead of visiting each (C4: the
      // spans outside their time range at a tile)
      uint64_t skip = lmask | ballot(((cmask >> lane) & 1) && (j_l >= len_l || (!RATE && j_l == 0)));
      if (INT_FAST) {
        const bool fc_l = ((cmask >> lane) & 1) && (j_l == 0 || j_l >= len_l || im_l != UINT32_MAX);
        skip |= ballot(fc_l);
        const uint64_t work = ballot(fc_l && j_l > 0 && j_l < len_l);
        if (work) {
          const uint32_t d_l = x_l.y - x_l.x;
          const uint32_t tl32 = gv ? (uint32_t)tl : (uint32_t)t_first;  // (x0 < t_first <= t < x1)
          if (AGG == 0 || AGG == 3) {
            uint64_t ysum = 0, qsum = 0;
            for (uint64_t m = work; m; m &= m - 1) {
              const int i = (int)__builtin_ctzll(m);
              const uint32_t x0 = readlane_u32(x_l.x, i), d = readlane_u32(d_l, i), im = readlane_u32(im_l, i);
              const double magr = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(magr_l), i));
              ysum += readlane_u64((uint64_t)y_l.x, i);
              const uint32_t u = tl32 - x0, mag = im & 0x7fffffffu;
              uint32_t q = (uint32_t)((double)u * magr);
              const int64_t rem = (int64_t)((uint64_t)u * mag) - (int64_t)((uint64_t)q * d);
              q = rem < 0 ? q - 1u : (rem >= (int64_t)d ? q + 1u : q);
              qsum = (im >> 31) ? qsum - q : qsum + q;
            }
            acc.ia = (int64_t)((acc.cnt == 0 ? 0ull : (uint64_t)acc.ia) + ysum + qsum);
            acc.cnt += (uint32_t)__popcll(work);
          } else {
            for (uint64_t m = work; m; m &= m - 1) {
              const int i = (int)__builtin_ctzll(m);
              const uint32_t x0 = readlane_u32(x_l.x, i), d = readlane_u32(d_l, i), im = readlane_u32(im_l, i);
              const double magr = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(magr_l), i));
              const int64_t y0 = (int64_t)readlane_u64((uint64_t)y_l.x, i);
              acc_push<AGG, MODE>(acc, lerp_long_prepped(tl32 - x0, d, y0, im, magr), 0.0);
            }
          }
        }
        // ... and the spans with one point x_n in the tile (smask), their
        // brackets prepared: each lane picks its bracket, (j-1, j) before x_n
        // or (j, j+1) after it (y_n on it), so one lerp a lane instead of the
        // ordered loop's divergent branches; the cursors move past x_n
        // lane-parallel afterwards (SpanGroup.java:702-784)
        const bool sf_l = ((smask >> lane) & 1) && (j_l == 0 || im_l != UINT32_MAX) &&
                          (j_l + 1 >= len_l || im2_l != UINT32_MAX);
        const uint64_t sfm = ballot(sf_l);
        if (sfm) {
          skip |= sfm;
          const uint32_t tl32 = gv ? (uint32_t)tl : (uint32_t)t_first;
          uint64_t lsum = 0;
          uint32_t lcnt = 0;
          for (uint64_t m = sfm; m; m &= m - 1) {
            const int i = (int)__builtin_ctzll(m);
            const uint32_t j = readlane_u32(j_l, i), len = readlane_u32(len_l, i);
            const uint32_t xc = readlane_u32(x_l.x, i), xn = readlane_u32(x_l.y, i), x2 = readlane_u32(x2_l, i);
            const uint32_t im = readlane_u32(im_l, i), im2 = readlane_u32(im2_l, i);
            const int64_t yc = (int64_t)readlane_u64((uint64_t)y_l.x, i), yn = (int64_t)readlane_u64((uint64_t)y_l.y, i);
            const double mr = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(magr_l), i));
            const double mr2 = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(magr2_l), i));
            const bool before = tl32 < xn, at = tl32 == xn;
            const bool act = gv && (before ? j > 0 : (at || j + 1 < len));
            const bool lerp = act && !at;
            const uint32_t a = before ? xc : xn, d = before ? xn - xc : x2 - xn, imv = before ? im : im2;
            const double mrv = lerp ? (before ? mr : mr2) : 0.0;
            const uint32_t u = lerp ? tl32 - a : 0u, mag = imv & 0x7fffffffu;
            uint32_t q = (uint32_t)((double)u * mrv);
            const int64_t rem = (int64_t)((uint64_t)u * mag) - (int64_t)((uint64_t)q * d);
            q = rem < 0 ? q - 1u : (rem >= (int64_t)d ? q + 1u : q);
            const int64_t v = at ? yn : ladd(before ? yc : yn, (imv >> 31) ? -(int64_t)q : (int64_t)q);
            if (AGG == 0 || AGG == 3) {
              lsum += act ? (uint64_t)v : 0ull;
              lcnt += act ? 1u : 0u;
            } else {
              acc_push_if<AGG, MODE>(acc, act, v, 0.0);
            }
          }
          if (AGG == 0 || AGG == 3) {
            acc.ia = (int64_t)((acc.cnt == 0 ? 0ull : (uint64_t)acc.ia) + lsum);
            acc.cnt += lcnt;
          }
          if (sf_l) {  // the cursor past point j
            j_l = j_l + 1;
            x_l = make_uint2(x_l.y, x2_l);
            y_l = make_longlong2(y_l.y, y2_l);
            f_l = 4u | ((f_l & 2u) ? 1u : 0u) | (f2_l ? 2u : 0u);
            dirty_l = true;
          }
        }
      }
      // Double sum / avg outside EXACT_ORDER, every lane's t on the double
      // path (dual mode: no long lerp is read): the one-point-in-tile spans
      // (C4: the bulk of what LIN leaves) the same way, from their prepared
      // doubles (y0, y1 - y0, 1 / (x1 - x0)) and the double of y_n; finite
      // brackets only. The order of the adds changes as LIN's does.
      constexpr bool DBL_FAST = (MODE == MODE_DBL || MODE == MODE_DUAL) && !RATE && (AGG == 0 || AGG == 3);
      if (DBL_FAST && !r.exact && (MODE == MODE_DBL || dual_all_dbl)) {
        const bool more_l = j_l + 1 < len_l;
        const double ynd_l = to_double(y_l.y, MODE == MODE_DBL || (f_l & 2u));
        const bool sf_l = ((smask >> lane) & 1) && (j_l == 0 || (x_l.y > x_l.x && __builtin_isfinite(y0d_l) &&
                                                                 __builtin_isfinite(dyd_l))) &&
                          __builtin_isfinite(ynd_l) &&
                          (!more_l || (__builtin_isfinite(y0d2_l) && __builtin_isfinite(dyd2_l)));
        const uint64_t sfm = ballot(sf_l);
        if (sfm) {
          skip |= sfm;
          const uint32_t tl32 = gv ? (uint32_t)tl : (uint32_t)t_first;
          double lsum = 0.0;
          uint32_t lcnt = 0;
          for (uint64_t m = sfm; m; m &= m - 1) {
            const int i = (int)__builtin_ctzll(m);
            const uint32_t j = readlane_u32(j_l, i), len = readlane_u32(len_l, i);
            const uint32_t xc = readlane_u32(x_l.x, i), xn = readlane_u32(x_l.y, i);
            const bool before = tl32 < xn, at = tl32 == xn;
            const bool act = gv && (before ? j > 0 : (at || j + 1 < len));
            auto rl = [&](double x) { return __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(x), i)); };
            const double y0a = rl(y0d_l), dya = rl(dyd_l), ria = rl(rinv_l);
            const double y0b = rl(y0d2_l), dyb = rl(dyd2_l), rib = rl(rinv2_l), yn = rl(ynd_l);
            const double v = at ? yn
                                : (before ? y0a + ((double)(tl32 - xc) * dya) * ria
                                          : y0b + ((double)(tl32 - xn) * dyb) * rib);
            lsum += act ? v : 0.0;
            lcnt += act ? 1u : 0u;
          }
          if (gv && lcnt) {
            acc.da = acc.cnt == 0 ? lsum : acc.da + lsum;
            acc.cnt += lcnt;
          }
          if (sf_l) {  // the cursor past point j
            j_l = j_l + 1;
            x_l = make_uint2(x_l.y, x2_l);
            y_l = make_longlong2(y_l.y, y2_l);
            f_l = 4u | ((f_l & 2u) ? 1u : 0u) | (f2_l ? 2u : 0u);
            dirty_l = true;
          }
        }
      }
      // A span with no point in this tile (its next point j lies past t_last):
      // every lane's bracket is (j-1, j), all from the cache (the span's lane
      // i of the batch registers above; only what the lerp reads is broadcast).
      auto cached = [&](uint32_t i) {
        const uint32_t j = readlane_u32(j_l, (int)i), len = readlane_u32(len_l, (int)i);
        if (!gv || j >= len) return;  // expired (all points consumed before this tile)
        if (RATE) {  // cur = j-1 (j >= 1), constant over the tile; active: tl <= last
          if (len >= 2)
            acc_push<AGG, MODE>(acc, 0, __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(rv_l), (int)i)));
          return;
        }
        if (j == 0) return;  // not started (F* covers the float look-ahead)
        const uint32_t f = readlane_u32(f_l, (int)i);
        const bool fc = (f & 1u) != 0, fn = (f & 2u) != 0;
        if (MODE == MODE_DUAL && (fc || fn)) acc.flag |= 1u;
        const uint32_t x0 = readlane_u32(x_l.x, (int)i);
        const uint32_t u = (uint32_t)(tl - (int64_t)x0);  // 0 < u < x1 - x0
        int64_t yi = 0;
        double yd = 0.0;
        if (need_long(fc, fn)) {
          const uint32_t x1 = readlane_u32(x_l.y, (int)i);
          const int64_t y0 = (int64_t)readlane_u64((uint64_t)y_l.x, (int)i);
          const uint32_t im = readlane_u32(im_l, (int)i);
          if (im != UINT32_MAX) {
            const double magr = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(magr_l), (int)i));
            yi = lerp_long_prepped(u, x1 - x0, y0, im, magr);
          } else {
            yi = lerp_long(tl, (int64_t)x0, y0, (int64_t)x1, (int64_t)readlane_u64((uint64_t)y_l.y, (int)i));
          }
        }
        if (MODE != MODE_INT) {
          // y0 + ((double)(t - x0) * (y1 - y0)) / (double)(x1 - x0), with y0 and
          // y1 - y0 converted once per batch; outside TSDBHIP_EXACT_ORDER the
          // division is a product with the batch-computed reciprocal (<= 1 ulp)
          const double y0d = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(y0d_l), (int)i));
          const double dyd = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(dyd_l), (int)i));
          const double num = (double)u * dyd;
          if (r.exact) {
            yd = y0d + num / (double)(readlane_u32(x_l.y, (int)i) - x0);
          } else {
            yd = y0d + num * __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(rinv_l), (int)i));
          }
        }
        acc_push<AGG, MODE>(acc, yi, yd);
      };
      for (uint32_t i = 0; i < nb;) {
        if ((skip >> i) & 1) {  // (added above)
          const uint64_t m = ~(skip >> i);
          i = min(nb, i + (m ? (uint32_t)__builtin_ctzll(m) : 64u));
          continue;
        }
        if ((dsingle >> i) & 1) {
          // a run of single-row direct spans with this span's width and type
          const uint32_t info0 = readlane_u32(dinfo_l, (int)i);
          const uint64_t m = ballot(dl && !(dinfo_l & 8u) && dinfo_l == info0) >> i;
          const uint32_t run = min(8u, ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m));
          if (info0 & 4u) {
            if (info0 & 2u) direct_run<AGG, MODE, RATE, 8, true>(r, acc, run, i, dvo_l, dga_l, dn_l, dx0_l, dstep_l, g, gv);
            else direct_run<AGG, MODE, RATE, 8, false>(r, acc, run, i, dvo_l, dga_l, dn_l, dx0_l, dstep_l, g, gv);
          } else {
            if (info0 & 2u) direct_run<AGG, MODE, RATE, 4, true>(r, acc, run, i, dvo_l, dga_l, dn_l, dx0_l, dstep_l, g, gv);
            else direct_run<AGG, MODE, RATE, 4, false>(r, acc, run, i, dvo_l, dga_l, dn_l, dx0_l, dstep_l, g, gv);
          }
          i += run;
          continue;
        }
        if (DONLY || ((dmask >> i) & 1)) {
          direct_one(kb + i, readlane_u32(dinfo_l, (int)i), readlane_u32(dga_l, (int)i), readlane_u32(dn_l, (int)i),
                     readlane_u64(dvo_l, (int)i));
          i++;
          continue;
        }
        if (ALIGNED_OK && ((almask >> i) & 1)) {
          const uint64_t m = almask >> i;  // bit 0: span kb + i
          constexpr uint32_t AR = 8;  // aligned spans whose values are in flight together (16: 3 waves/SIMD)
          const uint32_t run = min(AR, ~m == 0 ? 64u : (uint32_t)__builtin_ctzll(~m));
          int64_t v[AR];
#pragma unroll
          for (uint32_t u = 0; u < AR; u++) {
            const uint64_t eo_u = readlane_u64(eo_l, (int)min(i + u, 63u));
            v[u] = (u < run && gv) ? r.e_val[eo_u + g0 + lane] : 0;
          }
#pragma unroll
          for (uint32_t u = 0; u < AR; u++) {
            if (u >= run) break;
            if (gv) acc_push<AGG, MODE>(acc, v[u], MODE == MODE_INT ? 0.0 : to_double(v[u], true));
          }
          // cursor past the tile; cache stale (refilled by the general path)
          if ((uint32_t)lane >= i && (uint32_t)lane < i + run) { j_l = (uint32_t)(g0 + nvalid); f_l = 0; dirty_l = true; }
          i += run;
          continue;
        }
        if ((smask >> i) & 1) {
          // one point (x_n = point j) inside the tile: lanes before it keep the
          // cached bracket (j-1, j), the lane on it takes y_j, lanes after it
          // bracket (j, j+1) (SpanGroup.java:702-784)
          const uint32_t j = readlane_u32(j_l, (int)i), len = readlane_u32(len_l, (int)i);
          const uint32_t f = readlane_u32(f_l, (int)i), f2 = readlane_u32(f2_l, (int)i);
          const int64_t xc = (int64_t)readlane_u32(x_l.x, (int)i), xn = (int64_t)readlane_u32(x_l.y, (int)i);
          const int64_t x2 = (int64_t)readlane_u32(x2_l, (int)i);
          const int64_t yc = (int64_t)readlane_u64((uint64_t)y_l.x, (int)i), yn = (int64_t)readlane_u64((uint64_t)y_l.y, (int)i);
          const int64_t y2 = (int64_t)readlane_u64((uint64_t)y2_l, (int)i);
          const bool fc = (f & 1u) != 0, fn = (f & 2u) != 0, ff = f2 != 0;
          const bool more = j + 1 < len;  // point j+1 exists (past the tile)
          double rvn = 0.0;                // rate value at point j (j >= 1 in rate mode)
          if (RATE) rvn = (to_double(yn, fn) - to_double(yc, fc)) / (double)(xn - xc);
          if (gv) {
            if (RATE) {
              const double rvc = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(rv_l), (int)i));
              if (tl < xn) acc_push<AGG, MODE>(acc, 0, rvc);
              else if (more || tl == xn) acc_push<AGG, MODE>(acc, 0, rvn);  // else past the last point
            } else if (tl < xn) {
              if (j == 0) {  // not started: the next slot holds e_0
                if (MODE == MODE_DUAL && fn) acc.flag |= 1u;
              } else {
                if (MODE == MODE_DUAL && (fc || fn)) acc.flag |= 1u;
                int64_t yi = 0;
                double yd = 0.0;
                if (need_long(fc, fn)) {
                  const uint32_t im = readlane_u32(im_l, (int)i);
                  if (im != UINT32_MAX)
                    yi = lerp_long_prepped((uint32_t)(tl - xc), (uint32_t)(xn - xc), yc, im,
                                           __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(magr_l), (int)i)));
                  else
                    yi = lerp_long(tl, xc, yc, xn, yn);
                }
                if (MODE != MODE_INT) {
                  if (r.exact)
                    yd = lerp_double(tl, xc, to_double(yc, MODE == MODE_DBL || fc), xn, to_double(yn, MODE == MODE_DBL || fn));
                  else  // (the cached bracket's prepared doubles, as `cached`)
                    yd = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(y0d_l), (int)i)) +
                         ((double)(uint32_t)(tl - xc) *
                          __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(dyd_l), (int)i))) *
                             __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(rinv_l), (int)i));
                }
                acc_push<AGG, MODE>(acc, yi, yd);
              }
            } else if (tl == xn) {
              if (MODE == MODE_DUAL && (fn || (more && ff))) acc.flag |= 1u;
              acc_push<AGG, MODE>(acc, yn, MODE == MODE_INT ? 0.0 : to_double(yn, MODE == MODE_DBL || fn));
            } else if (more) {
              if (MODE == MODE_DUAL && (fn || ff)) acc.flag |= 1u;
              int64_t yi = 0;
              double yd = 0.0;
              if (need_long(fn, ff)) {
                const uint32_t im = readlane_u32(im2_l, (int)i);
                if (im != UINT32_MAX)
                  yi = lerp_long_prepped((uint32_t)(tl - xn), (uint32_t)(x2 - xn), yn, im,
                                         __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(magr2_l), (int)i)));
                else
                  yi = lerp_long(tl, xn, yn, x2, y2);
              }
              if (MODE != MODE_INT) {
                if (r.exact)
                  yd = lerp_double(tl, xn, to_double(yn, MODE == MODE_DBL || fn), x2, to_double(y2, MODE == MODE_DBL || ff));
                else
                  yd = __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(y0d2_l), (int)i)) +
                       ((double)(uint32_t)(tl - xn) *
                        __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(dyd2_l), (int)i))) *
                           __longlong_as_double((long long)readlane_u64((uint64_t)__double_as_longlong(rinv2_l), (int)i));
              }
              acc_push<AGG, MODE>(acc, yi, yd);
            }
          }
          // the cursor moves past point j
          if (lane == (int)i) {
            j_l = j + 1;
            x_l = make_uint2((uint32_t)xn, (uint32_t)x2);
            y_l = make_longlong2(yn, y2);
            f_l = 4u | (fn ? 1u : 0u) | (ff ? 2u : 0u);
            rv_l = rvn;
            dirty_l = true;
          }
          i++;
          continue;
        }
        if ((cmask >> i) & 1) {
          cached(i);
          i++;
          continue;
        }
        {
          const uint64_t eo = readlane_u64(eo_l, (int)i);
          const uint32_t len = readlane_u32(len_l, (int)i);
          const uint32_t jn = general(kb + i, eo, len, readlane_u32(j_l, (int)i));
          // refill the cache for cursor jn: points jn-1 and jn (rate: the
          // rate value of jn-1, SpanGroup.java:741-755)
          uint2 x = make_uint2(0, UINT32_MAX);
          longlong2 y = make_longlong2(0, 0);
          double rv = 0.0;
          uint32_t f = 4u;
          if (jn >= 1) {
            x.x = r.e_ts[eo + jn - 1];
            y.x = r.e_val[eo + jn - 1];
            if (r.e_flt[eo + jn - 1]) f |= 1u;
          }
          if (jn < len) {
            x.y = r.e_ts[eo + jn];
            y.y = r.e_val[eo + jn];
            if (r.e_flt[eo + jn]) f |= 2u;
          }
          if (RATE && jn >= 1) {
            const double yc = to_double(y.x, (f & 1u) != 0);
            if (jn >= 2) {
              const int64_t xp = r.e_ts[eo + jn - 2];
              const double yp = to_double(r.e_val[eo + jn - 2], r.e_flt[eo + jn - 2] != 0);
              rv = (yc - yp) / (double)((int64_t)x.x - xp);
            } else {
              rv = yc / (double)(int64_t)x.x;  // Q5: prev = (0, 0)
            }
          }
          if (lane == (int)i) { j_l = jn; x_l = x; y_l = y; rv_l = rv; f_l = f; dirty_l = true; }
        }
        i++;
      }
      // write back the cursors and caches that changed
      if (dirty_l) {
        ptr[sl] = j_l;
        S_f[sl] = f_l;
        if (f_l & 4u) {
          S_x[sl] = x_l;
          S_y[sl] = y_l;
          if (RATE) S_rv[sl] = rv_l;
        }
      }
    }
    if (gv) acc_store<AGG, MODE>(r, (uint64_t)chunk * r.T + g, acc);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
}

template <int AGG, int MODE, bool RATE, bool DONLY>
__global__ void __launch_bounds__(256) k_reduce(ReduceArgs r) {
  extern __shared__ __align__(16) uint8_t red_lds[];
  uint8_t* w = (!DONLY && r.lds_state) ? red_lds + (threadIdx.x / WAVE) * red_lds_stride(r.spans_per_chunk, RATE) : nullptr;
  reduce_wave<AGG, MODE, RATE, DONLY>(r, (blockIdx.x * blockDim.x + threadIdx.x) / WAVE, w);
}
// The same for sum / min / max / avg held to 128 VGPRs (4 waves a SIMD
// instead of 3 for the dual / double modes' 137): C4's reduce 9.66 -> 8.69
// ms, same box; dev, which would spill, and a 5-wave cap (12.7 ms, spills)
// keep the plain kernel.
template <int AGG, int MODE, bool RATE, bool DONLY>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_reduce_w4(ReduceArgs r) {
  extern __shared__ __align__(16) uint8_t red_lds[];
  uint8_t* w = (!DONLY && r.lds_state) ? red_lds + (threadIdx.x / WAVE) * red_lds_stride(r.spans_per_chunk, RATE) : nullptr;
  reduce_wave<AGG, MODE, RATE, DONLY>(r, (blockIdx.x * blockDim.x + threadIdx.x) / WAVE, w);
}

// The uniform path's E variant (uniform_run): every kept span's E is G
// itself (the key's bucket sequence, k_ds_reg), so span k's value at grid
// point g is e_val[e_off[k] + g] — no cursor, bracket or grid rank
// (SpanGroup.java:702-784 with x_cur == t at every t). A wave per (tile of
// 64 grid points, chunk of spans) pushes its chunk's spans in span order,
// 8 spans' values in flight; the partials are k_reduce's ([n_chunks][T]).
template <int AGG, int MODE>
__global__ void __launch_bounds__(256) k_ug_reduce(ReduceArgs r) {
  const int lane = lane_id();
  const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) / WAVE);
  const uint64_t n_tiles = (r.T + WAVE - 1) / WAVE;
  if (wave >= n_tiles * r.n_chunks) return;
  const uint32_t chunk = wave % r.n_chunks;
  const uint64_t g = (uint64_t)(wave / r.n_chunks) * WAVE + lane;
  const bool gv = g < r.T;
  const uint32_t k0 = chunk * r.spans_per_chunk, k1 = min(r.n_kept, k0 + r.spans_per_chunk);
  Acc acc;
  acc_init(acc);
  acc.fastdiv = AGG == 4 && MODE != MODE_INT;
  constexpr uint32_t U = 8;
  for (uint32_t kb = k0; kb < k1; kb += WAVE) {
    const uint32_t nk = min((uint32_t)WAVE, k1 - kb);
    const uint64_t eo_l = (uint32_t)lane < nk ? r.e_off[kb + lane] : 0;
    for (uint32_t i = 0; i < nk; i += U) {
      int64_t v[U];
#pragma unroll
      for (uint32_t u = 0; u < U; u++) {
        const uint64_t eo = readlane_u64(eo_l, (int)min(i + u, (uint32_t)WAVE - 1));
        v[u] = (i + u < nk && gv) ? r.e_val[eo + g] : 0;
      }
#pragma unroll
      for (uint32_t u = 0; u < U; u++)
        if (i + u < nk && gv) acc_push<AGG, MODE>(acc, v[u], MODE == MODE_INT ? 0.0 : to_double(v[u], true));
    }
  }
  if (gv) acc_store<AGG, MODE>(r, (uint64_t)chunk * r.T + g, acc);
}

__global__ void k_chunk_flags(const uint32_t* d_info, uint32_t n_kept, uint32_t spc, uint32_t* chunk_e) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k < n_kept && !(d_info[k] & 1u)) chunk_e[k / spc] = 1u;
}

// ------------------------------------------------------------- finalize ---
// few chunks: one thread per t, chunks in order
template <int AGG, int MODE, bool RATE>
__global__ void __launch_bounds__(256) k_finalize_seq(ReduceArgs r, FinalArgs f) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= f.T) return;
  const uint64_t st = f.stride ? f.stride : f.T;
  Acc a;
  acc_load<AGG, MODE>(r, g, a);
  for (uint32_t c = 1; c < f.n_chunks; c++) {
    Acc b;
    acc_load<AGG, MODE>(r, (uint64_t)c * st + g, b);
    acc_merge<AGG, MODE>(a, b);
  }
  finalize_one<AGG, MODE, RATE>(f, g, a);
}

// many chunks: one block per t; 256 threads take contiguous chunk ranges,
// then an order-preserving tree.
template <int AGG, int MODE, bool RATE>
__global__ void __launch_bounds__(256) k_finalize_par(ReduceArgs r, FinalArgs f) {
  __shared__ Acc s_acc[256];
  const uint64_t g = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint32_t per = (f.n_chunks + 255) / 256;
  const uint32_t c0 = t * per, c1 = min(f.n_chunks, c0 + per);
  Acc a;
  acc_init(a);
  for (uint32_t c = c0; c < c1; c++) {
    Acc b;
    acc_load<AGG, MODE>(r, (uint64_t)c * f.T + g, b);
    acc_merge<AGG, MODE>(a, b);
  }
  s_acc[t] = a;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    if ((t % (2 * d)) == 0) {
      Acc x = s_acc[t];
      acc_merge<AGG, MODE>(x, s_acc[t + d]);
      s_acc[t] = x;
    }
    __syncthreads();
  }
  if (t == 0) finalize_one<AGG, MODE, RATE>(f, g, s_acc[0]);
}

// Many chunks at large T (C3: ~290 chunks x 3600 t): a block of 16 waves per
// 64 consecutive t, so every partial load is a coalesced row segment; wave w
// merges chunk range w in order, then the 16 wave results merge in order.
// FINAL: finalize into the output; else store to dst slot t (rank combine).
constexpr uint32_t COLW = 16;
template <int AGG, int MODE, bool RATE, bool FINAL>
__global__ void __launch_bounds__(64 * COLW) k_chunks_cols(ReduceArgs r, ReduceArgs dst, FinalArgs f, uint64_t T,
                                                        uint32_t n_chunks) {
  __shared__ Acc s_acc[COLW][WAVE];
  const int lane = lane_id();
  const uint32_t w = threadIdx.x / WAVE;
  const uint64_t g = (uint64_t)blockIdx.x * WAVE + lane;
  const uint32_t per = (n_chunks + COLW - 1) / COLW;
  const uint32_t c0 = min(n_chunks, w * per), c1 = min(n_chunks, c0 + per);
  Acc a;
  acc_init(a);
  if (g < T) {
    // 8 chunks' partials loaded before they are merged (in order): one memory
    // round trip per 8 chunks instead of one per chunk (C3: ~128 a wave)
    uint32_t c = c0;
    for (; c + 8 <= c1; c += 8) {
      Acc b[8];
#pragma unroll
      for (int u = 0; u < 8; u++) acc_load<AGG, MODE>(r, (uint64_t)(c + u) * T + g, b[u]);
#pragma unroll
      for (int u = 0; u < 8; u++) acc_merge<AGG, MODE>(a, b[u]);
    }
    for (; c < c1; c++) {
      Acc b;
      acc_load<AGG, MODE>(r, (uint64_t)c * T + g, b);
      acc_merge<AGG, MODE>(a, b);
    }
  }
  s_acc[w][lane] = a;
  __syncthreads();
  if (w == 0 && g < T) {
    for (uint32_t v = 1; v < COLW; v++) acc_merge<AGG, MODE>(a, s_acc[v][lane]);
    if (FINAL) finalize_one<AGG, MODE, RATE>(f, g, a);
    else acc_store<AGG, MODE>(dst, g, a);
  }
}

}  // namespace tsdb

namespace tsdb {
// Combines n_chunks partials per t (in chunk order) into dst slot g.
template <int AGG, int MODE>
__global__ void __launch_bounds__(256) k_combine_chunks(ReduceArgs src, ReduceArgs dst, uint64_t T,
                                                        uint32_t n_chunks) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= T) return;
  Acc a;
  acc_load<AGG, MODE>(src, g, a);
  for (uint32_t c = 1; c < n_chunks; c++) {
    Acc b;
    acc_load<AGG, MODE>(src, (uint64_t)c * T + g, b);
    acc_merge<AGG, MODE>(a, b);
  }
  acc_store<AGG, MODE>(dst, g, a);
}

// The same combine for many chunks (a shard's ~2048 partials per t at small
// T): one block per t, contiguous chunk ranges per thread, then the
// order-preserving tree of k_finalize_par, stored to dst slot g.
template <int AGG, int MODE>
__global__ void __launch_bounds__(256) k_combine_par(ReduceArgs src, ReduceArgs dst, uint64_t T,
                                                     uint32_t n_chunks) {
  __shared__ Acc s_acc[256];
  const uint64_t g = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint32_t per = (n_chunks + 255) / 256;
  const uint32_t c0 = t * per, c1 = min(n_chunks, c0 + per);
  Acc a;
  acc_init(a);
  for (uint32_t c = c0; c < c1; c++) {
    Acc b;
    acc_load<AGG, MODE>(src, (uint64_t)c * T + g, b);
    acc_merge<AGG, MODE>(a, b);
  }
  s_acc[t] = a;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    if ((t % (2 * d)) == 0) {
      Acc x = s_acc[t];
      acc_merge<AGG, MODE>(x, s_acc[t + d]);
      s_acc[t] = x;
    }
    __syncthreads();
  }
  if (t == 0) acc_store<AGG, MODE>(dst, g, s_acc[0]);
}
}  // namespace tsdb
