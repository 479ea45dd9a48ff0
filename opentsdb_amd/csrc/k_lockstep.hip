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
// 64 grid points: wave 0 runs them (lane = grid point, wf_push with the true
// division, bit-exact with k_reduce's span-ordered pass), waves 1-3 stream
// the values into LDS ahead of it — span k's 64 values are 512 contiguous
// bytes (cell g of every span sits at grid point g) — DEV_B spans a phase,
// double-buffered, so the chain waits on LDS, not on HBM round trips (the
// general pass kept 8 loads in flight a lane: 23.6 ms at 100k series). The
// producers prove the proposal as they stream: every qualifier is compared
// with (x0 + g step - base) << 4 | flags (as k_lockstep); a mismatch sets
// `broken` and the call runs again on the proven path.
constexpr uint32_t DEV_B = 96;  // spans a phase (32 loads in flight a producer lane)
template <uint32_t W>
__global__ void __launch_bounds__(256) k_ug_dev(const uint8_t* val, const uint64_t* vo, const uint8_t* qual,
                                               const uint64_t* qo, uint32_t q0, uint32_t* broken, uint32_t n_kept,
                                               uint64_t T, uint32_t* grid, uint32_t x0, uint32_t step, FinalArgs f) {
  __shared__ int64_t s_buf[2][DEV_B][WAVE];
  const uint32_t w = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lane = lane_id();
  const uint64_t g = (uint64_t)blockIdx.x * WAVE + lane;
  const bool gv = g < T;
  const uint64_t gc = gv ? g : T - 1;  // (loads stay inside the row)
  const uint32_t nph = (n_kept + DEV_B - 1) / DEV_B;
  // this lane's qualifier under the proposal (big-endian as loaded)
  const uint32_t qe = (q0 + (uint32_t)gc * (step << 4)) & 0xFFFFu;
  const uint32_t qexp = ((qe & 0xFFu) << 8) | (qe >> 8);
  uint32_t bad = 0;
  auto produce = [&](uint32_t ph, int b) {  // waves 1..3: spans ph * DEV_B + j, j = w - 1, w + 2, ...
    constexpr uint32_t PER = DEV_B / 3;
    int64_t v[PER];
    uint32_t q[PER];
#pragma unroll
    for (uint32_t i = 0; i < PER; i++) {
      const uint32_t k = min(ph * DEV_B + (w - 1) + 3 * i, n_kept - 1);
      const uint8_t* p = val + vo[k] + (uint64_t)W * gc;
      v[i] = W == 8 ? (int64_t)bswap64(*(const uint64_t*)p) : (int64_t)(int32_t)bswap32(*(const uint32_t*)p);
      q[i] = *(const uint16_t*)(qual + qo[k] + 2 * gc);
    }
#pragma unroll
    for (uint32_t i = 0; i < PER; i++) {
      s_buf[b][(w - 1) + 3 * i][lane] = v[i];
      bad |= q[i] ^ qexp;
    }
  };
  if (w > 0) produce(0, 0);
  __syncthreads();
  Welford st;
  wf_init(st);
  for (uint32_t ph = 0; ph < nph; ph++) {
    const int b = ph & 1;
    if (w > 0) {
      if (ph + 1 < nph) produce(ph + 1, b ^ 1);
    } else {
      const uint32_t nk = min(DEV_B, n_kept - ph * DEV_B);
      for (uint32_t j = 0; j < nk; j++) wf_push(st, (double)s_buf[b][j][lane]);
    }
    __syncthreads();
  }
  if (w > 0 && ballot(bad != 0) && lane == 0) atomicOr(broken, 1u);
  if (w == 0 && gv) {
    grid[g] = x0 + (uint32_t)g * step;
    Acc a;
    acc_init(a);
    a.cnt = n_kept;
    a.wi = st;
    finalize_one<4, MODE_INT, false>(f, g, a);
  }
}

}  // namespace tsdb
