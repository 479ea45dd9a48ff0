// k_lockstep.hip — the no-downsampling reduction of a lockstep group: every
// kept span one row whose cells sit at x0 + c*step for c = 0..n-1 with the
// same (x0, n, step), value width and type (C3: 1M counters written at the
// same 1 s cadence). Then (SpanGroup.java:510-608) the union grid G is that
// sequence (rate: from its second point), every span is active at every t of
// G, the SGIterator never interpolates (x == x0 at every emission time,
// :702-730), and the rate is each span's own constant-step difference
// (:741-755, no Q5 state: no t lies before a span's second point). The value
// at G[g] is the cross-series aggregate of cell g (rate: of cells g and g+1),
// in span order (Aggregators.java:76-243).
//
// k_direct_opt (k_direct.hip) proposes the group from three qualifiers a span
// (cells 0, 1 and n-1: the cadence, width and type); this kernel proves the
// proposal while it streams: every cell's qualifier is compared with
// (x0 + c*step - base) << 4 | flags as the values are read, one pass over the
// reference's bytes (2 B of qualifier + W B of value a point) instead of the
// direct path's qualifier scan followed by a value pass. A mismatch sets
// `broken`; the call's results are then discarded and the call runs again on
// the proven path (spangroup_run, TSDBHIP_PATH_DIRECT_REDO).
//
// Work unit: one wave = a tile of 512 grid points (8 consecutive points a
// lane: one 16-B qualifier load and 2 / 4 16-B value loads a span) x a chunk
// of spans, the spans streamed in order with the next span's loads in flight
// while the current one is accumulated. A block's four waves take four
// consecutive chunks of one tile and merge their states in chunk order
// through LDS, so the per-t partials [n_chunks / 4][T] (the layout of
// k_reduce, combined in chunk order by the same finalize / exchange) are a
// quarter of one a wave: C3's 2048 chunks x 3600 points x 21 B made the
// combine read 155 MB.
#pragma once
#include "dev_common.h"
#include "k_reduce.hip"

namespace tsdb {

constexpr uint32_t LS_TILE = 512;  // grid points a wave (8 a lane)
constexpr uint32_t LS_GROUP = 4;   // chunks a block (its waves), merged into one partial

// one lane's slot state as it crosses LDS for the block's merge
struct LsSlot {
  uint32_t cnt, flag, dhas, pad;
  int64_t ia;
  double da, wim, wiv, wdm, wdv;
};

struct LockstepArgs {
  const uint64_t* d_voff;  // [n_kept] value byte offset of the span's cell 0
  const uint64_t* d_qoff;  // [n_kept] qualifier byte offset of the span's cell 0
  const uint8_t* val;
  const uint8_t* qual;
  uint32_t n;              // cells a span
  uint32_t q0;             // qualifier of cell 0 (delta << 4 | flags), the same in every span
  uint32_t step;
  uint32_t spc;            // spans a chunk
  uint32_t n_tiles;
  uint32_t n_chunks;       // chunks of spc spans; a block's 4 waves take 4 consecutive ones
                           // of one tile and combine them in order (LS_GROUP partials a block)
  uint32_t* broken;        // [1] set when a qualifier differs from the proposal
  // (the uniform path: G written by chunk 0's waves, G[g] = x0 + (g + g_off) step)
  uint32_t* grid_out;
  uint32_t x0, g_off;
};

template <uint32_t W, bool FLT>
DEVI int64_t ls_bits(uint64_t raw) {
  if (W == 8) return (int64_t)bswap64(raw);
  const uint32_t u = bswap32((uint32_t)raw);
  if (FLT) return dbits((double)__uint_as_float(u));
  return (int64_t)(int32_t)u;
}

// One span's bytes for this lane: cells c0 .. c0+7 (values as 8 raw words,
// qualifiers as 4 dwords of big-endian pairs) and, rate, the cell after the
// tile (the last lane's next cell).
template <uint32_t W>
struct LsRaw {
  uint32_t v[2 * W];  // W = 8: 16 dwords; W = 4: 8 dwords
  uint32_t q[4];
  uint64_t nxt;
};

template <uint32_t W, bool RATE>
DEVI void ls_load(const LockstepArgs& L, uint32_t k, uint32_t c0, uint32_t tile_end, LsRaw<W>& o) {
  const uint64_t vo = L.d_voff[k], qo = L.d_qoff[k];  // (uniform: scalar loads)
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)(L.val + vo), 0, (int)(L.n * W), 0x00020000);
  // (buffer range checks are per dword: a range ending inside a dword would
  // zero the row's last qualifier with its neighbour's bytes; whole 16-B
  // groups instead, the bytes past the row are masked)
  const __amdgpu_buffer_rsrc_t rq =
      __builtin_amdgcn_make_buffer_rsrc((void*)(L.qual + qo), 0, (int)((2u * L.n + 15u) & ~15u), 0x00020000);
#pragma unroll
  for (uint32_t i = 0; i < W / 2; i++) {
    const auto x = __builtin_amdgcn_raw_buffer_load_b128(rv, (int)(c0 * W + 16u * i), 0, 0);
    o.v[4 * i] = x[0]; o.v[4 * i + 1] = x[1]; o.v[4 * i + 2] = x[2]; o.v[4 * i + 3] = x[3];
  }
  const auto y = __builtin_amdgcn_raw_buffer_load_b128(rq, (int)(2u * c0), 0, 0);
  o.q[0] = y[0]; o.q[1] = y[1]; o.q[2] = y[2]; o.q[3] = y[3];
  o.nxt = 0;
  if (RATE && tile_end < L.n) {  // (uniform) the cell after the tile: the last lane's cur of its 8th point
    const uint8_t* p = L.val + vo + (uint64_t)W * tile_end;
    o.nxt = W == 8 ? *(const uint64_t*)p : (uint64_t)*(const uint32_t*)p;
  }
}

template <int AGG, int MODE, bool RATE, uint32_t W, bool FLT>
__global__ void __launch_bounds__(256) k_lockstep(ReduceArgs r, LockstepArgs L) {
  __shared__ LsSlot s_x[LS_GROUP - 1][WAVE];
  const int lane = lane_id();
  // (uniform: the span loop's offsets and buffer descriptors stay scalar)
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const uint32_t tile = blockIdx.x % L.n_tiles, cg = blockIdx.x / L.n_tiles;
  const uint32_t chunk = cg * LS_GROUP + w;
  const uint32_t k0 = chunk * L.spc, k1 = min(r.n_kept, k0 + L.spc);
  const bool act = chunk < L.n_chunks && k0 < k1;  // (every wave reaches the block's merge)
  const uint32_t c0 = tile * LS_TILE + 8u * (uint32_t)lane;  // this lane's first grid point (and cell)
  const uint32_t tile_end = tile * LS_TILE + LS_TILE;
  const uint32_t n = L.n;
  // the qualifiers of cells c0 .. c0+7 under the proposal, as loaded (two
  // big-endian u16 a dword), and the cells of the row (c < n)
  uint32_t qexp[4], qmask[4];
  {
    const uint32_t s16 = L.step << 4;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const uint32_t ca = c0 + 2u * (uint32_t)j;
      const uint32_t qa = L.q0 + ca * s16, qb = qa + s16;  // (< 2^16 for every cell of the row)
      const uint32_t x = (qa & 0xFFFFu) | (qb << 16);
      qexp[j] = __builtin_amdgcn_perm(x, x, 0x02030001u);  // bytes (1, 0, 3, 2): big-endian halves
      qmask[j] = (ca < n ? 0x0000FFFFu : 0u) | (ca + 1 < n ? 0xFFFF0000u : 0u);
    }
  }
  const uint64_t T = r.T;
  const bool full = (uint64_t)tile_end <= T;  // (uniform) every point of the tile is in G
  bool valid[8];
#pragma unroll
  for (int i = 0; i < 8; i++) valid[i] = (uint64_t)(c0 + i) < T;
  // rate: (y_cur - y_prev) / step; a power-of-two step divides exactly as a
  // product with its exact reciprocal (same IEEE result)
  const uint32_t step = L.step;
  const bool p2 = (step & (step - 1)) == 0;
  const double rs = __builtin_amdgcn_ldexp(1.0, -(int)__builtin_ctz(step | (1u << 31)));
  const double sd = (double)step;

  Acc acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc_init(acc[i]);
  uint32_t bad = 0;

  auto process = [&](const LsRaw<W>& cur, uint32_t k) {
#pragma unroll
    for (int j = 0; j < 4; j++) bad |= (cur.q[j] ^ qexp[j]) & qmask[j];
    int64_t b[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint64_t raw = W == 8 ? ((uint64_t)cur.v[2 * i + 1] << 32) | cur.v[2 * i] : (uint64_t)cur.v[i];
      b[i] = ls_bits<W, FLT>(raw);
    }
    const uint32_t cnt = k - k0;  // values before this one, in every slot
    // dev (double path, Aggregators.java:219-238): every span is active at
    // every t, so the Welford count is the same in all eight slots: one
    // reciprocal a span (wf_push_rcp's) instead of one a value
    double wf_r = 0.0;
    if (AGG == 4 && MODE != MODE_INT && cnt > 0) {
      const double dn = (double)(cnt + 1);
      wf_r = __builtin_amdgcn_rcp(dn);
      wf_r = __builtin_fma(__builtin_fma(-dn, wf_r, 1.0), wf_r, wf_r);  // one Newton step
    }
    double y[8];
    if (RATE) {
      double d[9];
#pragma unroll
      for (int i = 0; i < 8; i++) d[i] = to_double(b[i], FLT);
      // cell c0 + 8: the next lane's first cell; the last lane's from `nxt`
      const uint64_t b8 = wave_shl1_u64((uint64_t)b[0], (uint64_t)ls_bits<W, FLT>(cur.nxt));
      d[8] = to_double((int64_t)b8, FLT);
      if (p2) {
#pragma unroll
        for (int i = 0; i < 8; i++) y[i] = (d[i + 1] - d[i]) * rs;
      } else {
#pragma unroll
        for (int i = 0; i < 8; i++) y[i] = (d[i + 1] - d[i]) / sd;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 8; i++) y[i] = MODE == MODE_INT ? 0.0 : to_double(b[i], FLT);
    }
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (!full && !valid[i]) continue;
      if (AGG == 4 && MODE != MODE_INT) {
        Welford& w = acc[i].wd;
        if (cnt == 0) {
          w.mean = y[i];
          w.n = 1;
        } else {
          w.n++;
          const double dd = y[i] - w.mean;
          const double nm = __builtin_fma(dd, wf_r, w.mean);
          w.var += dd * (y[i] - nm);
          w.mean = nm;
        }
        acc[i].cnt++;
      } else {
        acc_push<AGG, MODE>(acc[i], RATE ? 0 : b[i], y[i]);
      }
    }
  };
  // two register sets: the next span's loads are in flight while one is
  // accumulated (the last span reloads itself, so the loads stay straight-line)
  if (act) {
    LsRaw<W> ra, rb;
    ls_load<W, RATE>(L, k0, c0, tile_end, ra);
    for (uint32_t k = k0;;) {
      ls_load<W, RATE>(L, min(k + 1, k1 - 1), c0, tile_end, rb);
      process(ra, k);
      if (++k >= k1) break;
      ls_load<W, RATE>(L, min(k + 1, k1 - 1), c0, tile_end, ra);
      process(rb, k);
      if (++k >= k1) break;
    }
    if (ballot(bad != 0) && lane == 0) atomicOr(L.broken, 1u);
    if (L.grid_out && chunk == 0) {
#pragma unroll
      for (int i = 0; i < 8; i++)
        if (valid[i]) L.grid_out[c0 + i] = L.x0 + (c0 + (uint32_t)i + L.g_off) * L.step;
    }
  }
  // the block's chunks merged in chunk order (span order), one slot at a time
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (w > 0) {
      LsSlot& x = s_x[w - 1][lane];
      x.cnt = acc[i].cnt; x.flag = acc[i].flag; x.dhas = acc[i].dhas;
      x.ia = acc[i].ia; x.da = acc[i].da;
      x.wim = acc[i].wi.mean; x.wiv = acc[i].wi.var; x.wdm = acc[i].wd.mean; x.wdv = acc[i].wd.var;
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (uint32_t j = 0; j < LS_GROUP - 1; j++) {
        const LsSlot& x = s_x[j][lane];
        Acc b;
        acc_init(b);
        b.cnt = x.cnt; b.flag = x.flag; b.dhas = x.dhas; b.ia = x.ia; b.da = x.da;
        b.wi.n = x.cnt; b.wi.mean = x.wim; b.wi.var = x.wiv;
        b.wd.n = x.cnt; b.wd.mean = x.wdm; b.wd.var = x.wdv;
        acc_merge<AGG, MODE>(acc[i], b);
      }
      if (valid[i]) acc_store<AGG, MODE>(r, (uint64_t)cg * T + c0 + i, acc[i]);
    }
    __syncthreads();
  }
}

// ---- integer dev of a lockstep group (no rate): the reference's sequential
// Welford over the spans in span order before the (long) truncation
// (Aggregators.java:196-237) admits no merge of partial states, so each grid
// point is one chain of n_kept dependent steps. A block holds the chains of
// GP grid points, 2 + UG_DEV_NP waves:
//   wave 0  the mean chains (lane = grid point): mean' = mean + (x - mean)/n,
//           each step's (x - mean, mean') to LDS;
//   wave 1  the M2 sums one phase behind: var += (x - mean) (x - mean'), in
//           span order (the same roundings as wf_push, dev_common.h);
//   waves 2+  stream the values into LDS ahead of them — span k's GP values
//           are W * GP contiguous bytes (cell g of every span sits at grid
//           point g), 64 / GP spans a load instruction — DEV_B spans a phase,
//           a software pipeline over UG_DEV_DEPTH = 3 register sets (values
//           of phase ph + 1 stored while those of ph + 4 and the row offsets
//           of ph + 7 load: three phases of latency for each level), and
//           convert them to double; they also prove the proposal as they
//           stream: every qualifier is compared with (x0 + g step - base) << 4
//           | flags (as k_lockstep); a mismatch sets `broken` and the call
//           runs again on the proven path.
// The chain's division (x - mean) / n is Markstein's correction of a product
// with r = RN(1/n): q0 = RN(d r), e = d - n q0 (exact, one fma), q = RN(q0 +
// e r) = RN(d / n) — the quotient of a double by an integer n never sits on a
// rounding midpoint and stays normal here — bit-exact with the division; r
// comes from the producers through LDS, n is converted by the chain wave
// (span 0 takes the same step from mean 0 with n = 1). The mean
// chain is then five dependent double operations a step on a SIMD of its own
// (round 6: 95 -> 56.7 ms for C3's 1M series, 9.5 -> 5.7 ms for 100k, with
// GP = 16: 225 blocks instead of 57, and the conversions off the chain; then
// 64-span phases 44.8 ms, the two-set producer pipeline 41.3 ms, the chain's
// LDS reads a group ahead (scheduling barrier) 39.8 ms, four producer waves
// 39.2 ms, three register sets 35.0 ms. Without the mean chain the kernel
// takes 25 ms.)
#ifndef UG_DEV_B
#define UG_DEV_B 64u  // (C3 1M series: 16 / 32 / 48 / 64 / 80 / 96 / 128 spans 73.7 / 55.2 / 48.4 / 44.8 / 57.0 / 56.7 / 57.7 ms)
#endif
#ifndef UG_DEV_U
#define UG_DEV_U 8u  // chain steps whose LDS reads are in flight together
#endif
#ifndef UG_DEV_DEPTH
#define UG_DEV_DEPTH 3u  // producer register sets (phases of load latency; 2 / 3: 39.2 / 35.0 ms)
#endif
#ifndef UG_DEV_AHEAD
#define UG_DEV_AHEAD 1u  // phases the producers store ahead of the chain
#endif
#ifndef UG_DEV_NP
#define UG_DEV_NP 4u  // producer waves (the block: 2 + UG_DEV_NP waves; C3 1M series 2 / 4: 39.8 / 39.2 ms)
#endif
constexpr uint32_t DEV_B = UG_DEV_B;  // spans a phase
#ifndef UG_DEV_ABL
#define UG_DEV_ABL 0
#endif
template <uint32_t W, uint32_t GP>
__global__ void __launch_bounds__(64 * (2 + UG_DEV_NP)) k_ug_dev(const uint8_t* val, const uint64_t* vo, const uint8_t* qual,
                                               const uint64_t* qo, uint32_t q0, uint32_t* broken, uint32_t n_kept,
                                               uint64_t T, uint32_t* grid, uint32_t x0, uint32_t step, FinalArgs f) {
  static_assert(GP == 16 || GP == 32 || GP == 64, "grid points a block");
  constexpr uint32_t SPL = WAVE / GP;  // spans a producer load instruction
  constexpr uint32_t NP = UG_DEV_NP;   // producer waves
  static_assert(DEV_B % (NP * SPL) == 0, "a phase's spans split over the producers");
  constexpr uint32_t AH = UG_DEV_AHEAD;  // phases the producers store ahead of the chain
  static_assert(AH == 1 || AH == 2, "store lead");
  constexpr uint32_t RB = AH + 2;        // the value ring: stored, (stored earlier,) chain, M2 sums
  __shared__ double s_buf[RB][DEV_B][GP];
  __shared__ double2 s_dm[2][DEV_B][GP];              // each step's (x - mean, mean')
  __shared__ double s_rcp[RB][DEV_B];                 // RN(1/n) (n = span index + 1)
  __shared__ double s_var[GP];
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lane = lane_id();
  const uint32_t gl = (uint32_t)lane % GP, si = (uint32_t)lane / GP;  // (producers: grid point, span of the load)
  const uint32_t gchain = w < 2 ? (uint32_t)lane : gl;
  const uint64_t g = (uint64_t)blockIdx.x * GP + gchain;
  const bool gv = g < T && gchain < GP;
  const uint64_t gc = g < T ? g : T - 1;  // (loads stay inside the row)
  const uint32_t nph = (n_kept + DEV_B - 1) / DEV_B;
  // this lane's qualifier under the proposal (big-endian as loaded)
  const uint32_t qe = (q0 + (uint32_t)gc * (step << 4)) & 0xFFFFu;
  const uint32_t qexp = ((qe & 0xFFu) << 8) | (qe >> 8);
  uint32_t bad = 0;
  constexpr uint32_t PER = DEV_B / (NP * SPL);  // load instructions a producer a phase
  // a producer's register set: the values of phase p and the row offsets of
  // phase p + 2 (two sets: values two phases ahead of their store, offsets two
  // phases ahead of their values)
  struct DevSet {
    int64_t v[PER];
    uint32_t q[PER];
    uint64_t ov[PER], oq[PER];
  };
  constexpr uint32_t D = UG_DEV_DEPTH;  // register sets: values D phases ahead of their store
  static_assert(D >= 2 && D <= 4, "pipeline depth");
  DevSet sa, sb, sc, sd;
  auto slot = [&](uint32_t i) { return (w - 2) * SPL + NP * SPL * i + si; };  // span slot of the phase
  auto load_offs = [&](DevSet& S, uint32_t ph) {  // (spans past the last: the last one's, never stored)
    if (UG_DEV_ABL == 2) return;
#pragma unroll
    for (uint32_t i = 0; i < PER; i++) {
      const uint32_t k = min(ph * DEV_B + slot(i), n_kept - 1);
      S.ov[i] = vo[k];
      S.oq[i] = qo[k];
    }
  };
  auto load_vals = [&](DevSet& S) {
    if (UG_DEV_ABL == 2) {
      for (uint32_t i = 0; i < PER; i++) { S.v[i] = (int64_t)i; S.q[i] = qexp; }
      return;
    }
#pragma unroll
    for (uint32_t i = 0; i < PER; i++) {
      const uint8_t* p = val + S.ov[i] + (uint64_t)W * gc;
      S.v[i] = W == 8 ? (int64_t)bswap64(*(const uint64_t*)p) : (int64_t)(int32_t)bswap32(*(const uint32_t*)p);
      S.q[i] = *(const uint16_t*)(qual + S.oq[i] + 2 * gc);
    }
  };
  auto store = [&](uint32_t ph, const DevSet& S) {  // phase ph's values, converted, and its counts
    if (w == 2)
      for (uint32_t j = (uint32_t)lane; j < DEV_B; j += WAVE) {
        const double dn = (double)(ph * DEV_B + j + 1);
        s_rcp[ph % RB][j] = 1.0 / dn;
      }
#pragma unroll
    for (uint32_t i = 0; i < PER; i++) {
      s_buf[ph % RB][slot(i)][gl] = (double)S.v[i];
      if (ph * DEV_B + slot(i) < n_kept) bad |= S.q[i] ^ qexp;
    }
  };
  if (w >= 2) {  // phase 0 stored; set i (of D): values of phase 1 + i, offsets of 1 + i + D
    load_offs(sa, 0);
    load_vals(sa);
    store(0, sa);
    if (AH == 2) {
      load_offs(sa, 1);
      load_vals(sa);
      store(1, sa);
    }
    load_offs(sa, AH);
    load_offs(sb, AH + 1);
    if (D >= 3) load_offs(sc, AH + 2);
    if (D >= 4) load_offs(sd, AH + 3);
    load_vals(sa);
    load_vals(sb);
    if (D >= 3) load_vals(sc);
    if (D >= 4) load_vals(sd);
    load_offs(sa, AH + D);
    load_offs(sb, AH + 1 + D);
    if (D >= 3) load_offs(sc, AH + 2 + D);
    if (D >= 4) load_offs(sd, AH + 3 + D);
  }
  __syncthreads();
  double mean = 0, var = 0;
  // one phase: the producers store phase ph + 1 from `cur` and refill it
  // (values of ph + 1 + D, offsets of ph + 1 + 2 D); wave 0 runs the chains
  // over phase ph, wave 1 the M2 sums over ph - 1
  auto phase = [&](uint32_t ph, DevSet& cur) {
    if (w >= 2) {
      if (ph + AH < nph) store(ph + AH, cur);
      if (ph + AH + D < nph) load_vals(cur);
      if (ph + AH + 2 * D < nph) load_offs(cur, ph + AH + 2 * D);
    } else if (w == 0 && ph < nph && (uint32_t)lane < GP && UG_DEV_ABL != 5) {  // the mean chains
      // (span 0 takes the same step from mean = 0 with n = 1: d = x, q = x
      // exactly, mean' = x — wf_push's first value — so no step is special)
      const uint32_t nk = min(DEV_B, n_kept - ph * DEV_B), b3 = ph % RB, b2 = ph & 1;
      const uint32_t base = ph * DEV_B + 1;  // n of the phase's first span
      auto chain_step = [&](uint32_t j, double x, double r) {
        const double dn = (double)(base + j);  // (exact: n < 2^32)
        const double d = x - mean;
        const double qa = d * r;
#if UG_DEV_ABL == 1  // (ablation builds only, wrong results: 1 the product without its correction,
                    // 2 no loads, 3 a one-add chain, 4 no M2 sums, 5 no mean chain)
        const double nm = mean + qa;
#elif UG_DEV_ABL == 3
        const double nm = mean + x;
#else
        const double e = __builtin_fma(-dn, qa, d);
        const double nm = mean + __builtin_fma(e, r, qa);
#endif
        s_dm[b2][j][lane] = make_double2(d, nm);
        mean = nm;
      };
      constexpr uint32_t U = UG_DEV_U;
      static_assert(DEV_B % U == 0, "chain groups");
      if (nk == DEV_B) {
        // a full phase, straight-line: the next U steps' LDS reads issued
        // before this group's chain (the scheduling barrier keeps them there;
        // without it the compiler sank each read next to its use, an LDS
        // latency on every step of the chain)
        double xa[U], ra[U];
        auto fetch = [&](uint32_t j0, double* x, double* r) {
#pragma unroll
          for (uint32_t u = 0; u < U; u++) {
            x[u] = s_buf[b3][j0 + u][lane];
            r[u] = s_rcp[b3][j0 + u];
          }
        };
        fetch(0, xa, ra);
        for (uint32_t j = 0; j < DEV_B; j += U) {
          double xb[U], rb[U];
          fetch(j + U < DEV_B ? j + U : j, xb, rb);  // (the last group re-reads itself)
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (uint32_t u = 0; u < U; u++) chain_step(j + u, xa[u], ra[u]);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (uint32_t u = 0; u < U; u++) {
            xa[u] = xb[u];
            ra[u] = rb[u];
          }
        }
      } else {  // the last, partial phase
        for (uint32_t j = 0; j < nk; j++) chain_step(j, s_buf[b3][j][lane], s_rcp[b3][j]);
      }
    } else if (w == 1 && ph >= 1 && (uint32_t)lane < GP && UG_DEV_ABL != 4) {  // the M2 sums of the phase before
      const uint32_t p = ph - 1, nk = min(DEV_B, n_kept - p * DEV_B), b3 = p % RB, b2 = p & 1;
      for (uint32_t j = p == 0 ? 1u : 0u; j < nk; j++) {
        const double2 dm = s_dm[b2][j][lane];
        var += dm.x * (s_buf[b3][j][lane] - dm.y);
      }
    }
    __syncthreads();
  };
  for (uint32_t ph = 0; ph <= nph; ph += D) {
    phase(ph, sa);
    if (ph + 1 <= nph) phase(ph + 1, sb);
    if (D >= 3 && ph + 2 <= nph) phase(ph + 2, sc);
    if (D >= 4 && ph + 3 <= nph) phase(ph + 3, sd);
  }
  if (w == 1 && (uint32_t)lane < GP) s_var[lane] = var;
  if (w >= 2 && ballot(bad != 0) && lane == 0) atomicOr(broken, 1u);
  __syncthreads();
  if (w == 0 && gv) {
    grid[g] = x0 + (uint32_t)g * step;
    Acc a;
    acc_init(a);
    a.cnt = n_kept;
    a.wi.n = n_kept;
    a.wi.mean = mean;
    a.wi.var = s_var[lane];
    finalize_one<4, MODE_INT, false>(f, g, a);
  }
}

}  // namespace tsdb
