// k_group.hip — group-by batching: the SpanGroups
// TsdbQuery.groupByAndAggregate builds for one query (TsdbQuery.java:294-363)
// evaluated in one call. Spans of group g are the contiguous span range
// [gss[g], gss[g+1]) (groups in ByteMap order, spans in TreeMap order within a
// group). Per-span work (assembly, decode, downsampling) runs once over every
// span; the union grid is segmented: group g owns bitmap words
// [wbase[g], wbase[g] + nw[g] + 1) over its own [lo[g], hi[g]] (the last word
// is a zero pad, whose rank is T_g), and its grid points are
// grid[goff[g], goff[g] + T_g).
#pragma once
#include "dev_common.h"
#include "k_grid.hip"
#include "k_reduce.hip"
#include "k_direct.hip"

namespace tsdb {

// Per-group results of the segmented passes (one 64-B slot per group).
struct GroupDev {
  unsigned long long fstar;   // F* of the group (max float-first ts + 1, 0: none)
  unsigned long long nan_t;   // first NaN/Inf output index (finalize)
  unsigned long long bad_at;  // lazy illegal-cell index << 4 | code
  uint64_t goff;              // first grid index of the group
  uint64_t T;                 // |G_g|
  uint32_t gfl;               // bit0: some E point is a float, bit1: some is an int
  uint32_t reserved;
  uint64_t pad[2];
};

__global__ void k_group_init(GroupDev* gd, uint32_t n_groups) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  GroupDev z = {};
  z.nan_t = ~0ull;
  z.bad_at = ~0ull;
  gd[g] = z;
}

// Per-group span statistics after assembly (SpanGroup.java:135-141 keep rule
// applied per span by k_assemble).
struct GroupStat {
  uint64_t k0;       // first kept index of the group
  uint64_t nk;       // kept spans
  uint64_t n_input;  // SpanGroup.aggregatedSize() (SpanGroup.java:206-212)
  int64_t first;     // min first ts of the kept spans
  int64_t last;      // max last ts of the kept spans
};

// Block per group (grid-stride): kept-span group ids and the group's stats.
__global__ void __launch_bounds__(256) k_group_stats(const uint32_t* gss, uint32_t n_groups, uint32_t n_spans,
                                                     uint32_t n_kept, const uint8_t* sp_kept, const uint64_t* kidx,
                                                     const uint32_t* sp_ncells, const int64_t* sp_first,
                                                     const int64_t* sp_last, uint32_t* kgrp, GroupStat* stat) {
  __shared__ uint64_t sh_c[4], sh_n[4];
  __shared__ int64_t sh_f[4], sh_l[4];
  for (uint32_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
    const uint32_t s0 = gss[g], s1 = gss[g + 1];
    uint64_t cnt = 0, nk = 0;
    int64_t f = INT64_MAX, l = INT64_MIN;
    for (uint32_t s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
      if (!sp_kept[s]) continue;
      kgrp[kidx[s]] = g;
      nk++;
      cnt += sp_ncells[s];
      f = min(f, sp_first[s]);
      l = max(l, sp_last[s]);
    }
    auto add = [](uint64_t x, uint64_t y) { return x + y; };
    cnt = block_reduce_256(cnt, add, sh_c);
    nk = block_reduce_256(nk, add, sh_n);
    f = block_reduce_256(f, [](int64_t x, int64_t y) { return min(x, y); }, sh_f);
    l = block_reduce_256(l, [](int64_t x, int64_t y) { return max(x, y); }, sh_l);
    if (threadIdx.x == 0) {
      GroupStat st;
      st.k0 = s0 < n_spans ? kidx[s0] : n_kept;
      st.nk = nk;
      st.n_input = cnt;
      st.first = f;
      st.last = l;
      stat[g] = st;
    }
    __syncthreads();
  }
}

// Wave per kept span, after decode: E_EMPTY_SPAN (SpanGroup.java:452-455),
// the group's F* and (flags) whether the group's E holds floats / ints —
// what k_span_summary and the decode kernels' global flags give one group.
// Direct spans (d_info & DIR_ON, k_direct.hip) hold no E: one cell type,
// first point x0.
__global__ void __launch_bounds__(256) k_group_summary(const uint64_t* e_off, const uint32_t* e_len,
                                                       const uint32_t* e_ts, const uint8_t* e_flt, uint32_t n_kept,
                                                       int32_t rate, int32_t flags, const uint32_t* kgrp,
                                                       const uint32_t* d_info, const uint32_t* d_x0,
                                                       GroupDev* gd, unsigned long long* err) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  for (uint32_t k = wave; k < n_kept; k += nwaves) {
    const uint32_t len = e_len[k];
    const uint64_t eo = e_off[k];
    GroupDev* g = &gd[kgrp[k]];
    const uint32_t info = d_info ? d_info[k] : 0u;
    if (info & DIR_ON) {
      if (lane == 0) {
        const bool f = (info & DIR_FLT) != 0;
        if (f && !rate) {
          const unsigned long long fs = (unsigned long long)d_x0[k] + 1;
          if (g->fstar < fs) atomicMax(&g->fstar, fs);
        }
        const uint32_t bits = f ? 1u : 2u;
        if (flags && (g->gfl & bits) != bits) atomicOr(&g->gfl, bits);
      }
      continue;
    }
    if (len == 0) {
      if (lane == 0) err_raise(err, 1, 0, -3 /*E_EMPTY_SPAN*/);
      continue;
    }
    if (lane == 0 && !rate && e_flt[eo]) {
      const unsigned long long fs = (unsigned long long)e_ts[eo] + 1;  // +1: 0 = none
      if (g->fstar < fs) atomicMax(&g->fstar, fs);
    }
    if (!flags) continue;
    bool f = false, i = false;
    for (uint32_t j = lane; j < len; j += WAVE) {
      const bool x = e_flt[eo + j] != 0;
      f |= x;
      i |= !x;
    }
    const uint32_t bits = (ballot(f) ? 1u : 0u) | (ballot(i) ? 2u : 0u);
    if (lane == 0 && (g->gfl & bits) != bits) atomicOr(&g->gfl, bits);
  }
}

// Geometry of the segmented bitmap, per group (device copies of host math).
struct GroupGrid {
  const int64_t* lo;      // [G]
  const int64_t* hi;      // [G] (lo > hi: empty grid)
  const uint64_t* wbase;  // [G] first word
  const uint32_t* nw;     // [G] words (without the pad word)
  const uint32_t* wgrp;   // [W] group of each word
};

// Block per group: the word -> group map.
__global__ void __launch_bounds__(256) k_group_words(GroupGrid q, uint32_t n_groups, uint32_t* wgrp) {
  for (uint32_t g = blockIdx.x; g < n_groups; g += gridDim.x) {
    const uint64_t b = q.wbase[g];
    const uint32_t n = q.nw[g] + 1;
    for (uint32_t w = threadIdx.x; w < n; w += blockDim.x) wgrp[b + w] = g;
  }
}

// k_grid_mark over every kept span, each into its group's bitmap.
// (direct candidates, which hold no E, are marked by k_direct_mark_seg)
__global__ void __launch_bounds__(256) k_grid_mark_seg(const uint64_t* e_off, const uint32_t* e_len,
                                                       const uint32_t* e_ts, uint32_t n_kept, int32_t rate,
                                                       const uint32_t* kgrp, GroupGrid q, uint32_t* bitmap,
                                                       const uint32_t* d_info) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  for (uint32_t k = wave; k < n_kept; k += nwaves) {
    if (d_info && (d_info[k] & DIR_ON)) continue;
    const uint32_t g = kgrp[k];
    const int64_t lo = q.lo[g], hi = q.hi[g];
    if (lo > hi) continue;
    uint32_t* bm = bitmap + q.wbase[g];
    const uint64_t eo = e_off[k];
    const uint32_t len = e_len[k];
    for (uint32_t i0 = rate ? 1 : 0; i0 < len; i0 += WAVE) {
      const uint32_t i = i0 + lane;
      if (i >= len) break;
      const int64_t t = e_ts[eo + i];
      if (t > hi) break;  // sorted: the rest are beyond end
      if (t < lo) continue;
      const uint64_t b = (uint64_t)(t - lo);
      const uint32_t bit = 1u << (b & 31);
      uint32_t* w = &bm[b >> 5];
      if (!(*w & bit)) atomicOr(w, bit);
    }
  }
}

// k_grid_emit over the concatenated bitmaps: global ranks, grid points from
// each word's own group origin.
__global__ void __launch_bounds__(256) k_grid_emit_seg(uint32_t* bitmap, uint32_t* word_rank,
                                                       const uint32_t* block_sum, uint64_t nwords, GroupGrid q,
                                                       uint32_t* grid) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= nwords) return;
  const uint32_t r = word_rank[w] + block_sum[w >> 10];
  word_rank[w] = r;
  const uint32_t g = q.wgrp[w];
  const int64_t base = q.lo[g] + (int64_t)((w - q.wbase[g]) * 32);
  uint32_t bits = bitmap[w];
  uint32_t i = r;
  while (bits) {
    const int b = __builtin_ctz(bits);
    grid[i++] = (uint32_t)(base + b);
    bits &= bits - 1;
  }
}

// Thread per group: grid offset and size from the global word ranks.
__global__ void k_group_T(GroupGrid q, uint32_t n_groups, const uint32_t* word_rank, GroupDev* gd) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n_groups) return;
  const uint64_t b = q.wbase[g];
  const uint32_t r0 = word_rank[b], r1 = word_rank[b + q.nw[g]];  // pad word: rank after the group
  gd[g].goff = r0;
  gd[g].T = r1 - r0;
}

// Word ranks relative to the group (what grid_rank expects per group).
__global__ void __launch_bounds__(256) k_group_rebase(GroupGrid q, uint64_t nwords, const GroupDev* gd,
                                                      uint32_t* word_rank) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= nwords) return;
  word_rank[w] -= (uint32_t)gd[q.wgrp[w]].goff;
}

// k_bad_index per kept span against its group's grid.
__global__ void k_bad_index_seg(const int64_t* e_bad, const uint64_t* e_off, const uint32_t* e_ts,
                                uint32_t n_kept, int32_t rate, const uint32_t* kgrp, GroupGrid q,
                                const uint32_t* bitmap, const uint32_t* word_rank, GroupDev* gd) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_kept) return;
  const int64_t b = e_bad[k];
  if (b < 0) return;
  const uint32_t g = kgrp[k];
  const uint64_t idx = (uint64_t)(b >> 4), code = (uint64_t)(b & 15);
  uint64_t at;
  if (idx == 0 || (rate && idx == 1)) {
    at = 0;
  } else {
    const int64_t tp = e_ts[e_off[k] + idx - 1];
    if (tp > q.hi[g]) return;  // never consumed
    const uint64_t wb = q.wbase[g];
    at = gd[g].T == 0 ? 0 : grid_rank(bitmap + wb, word_rank + wb, q.lo[g], tp);
  }
  atomicMin(&gd[g].bad_at, (unsigned long long)((at << 4) | code));
}

// ---- one reduce launch for many groups ------------------------------------
// Per-group view of the shared E / grid / partial buffers (host-computed
// after the segmented grid is known).
struct SegGroup {
  uint64_t k0;       // first kept index
  uint64_t goff;     // first grid index (output offset)
  uint64_t T;        // |G_g|
  uint64_t wbase;    // first bitmap word
  int64_t lo;        // bitmap origin
  uint64_t fstar;    // F*_g
  uint64_t poff;     // partials offset ([n_chunks][T] block of the group)
  uint64_t coff;     // cursor / bracket-cache offset
  uint64_t choff;    // chunk offset (chunk_e)
  uint32_t nk, spc, n_chunks, tpw, ntg, mode;
};

struct SegReduce {
  const SegGroup* sg;
  const uint32_t* glist;     // groups of this launch (one reduce mode)
  const uint64_t* wv_start;  // [n+1] first wave of each listed group
  uint32_t n;
};

DEVI void seg_view(ReduceArgs& r, const SegGroup& G) {
  r.e_off += G.k0;
  r.e_len += G.k0;
  r.kept += G.k0;
  r.n_kept = G.nk;
  r.grid += G.goff;
  r.T = G.T;
  r.bitmap += G.wbase;
  r.word_rank += G.wbase;
  r.lo = G.lo;
  r.spans_per_chunk = G.spc;
  r.n_chunks = G.n_chunks;
  r.tiles_per_wave = G.tpw;
  r.n_tile_groups = G.ntg;
  r.fstar = G.fstar;
  if (r.d_info) {
    r.d_info += G.k0;
    r.d_n += G.k0;
    r.d_ga += G.k0;
    r.d_voff += G.k0;
    r.d_x0 += G.k0;
    r.d_step += G.k0;
    r.d_c0 += G.k0;
    r.d_r0 += G.k0;
    r.chunk_e += G.choff;
  }
  r.ptr += G.coff;
  r.st_x += G.coff;
  r.st_y += G.coff;
  r.st_rv += G.coff;
  r.st_f += G.coff;
  r.p_cnt += G.poff;
  r.p_flag += G.poff;
  r.p_i += G.poff;
  r.p_d += G.poff;
  r.p_dhas += G.poff;
  if (r.p_wim) {
    r.p_wim += G.poff;
    r.p_wiv += G.poff;
    r.p_wdm += G.poff;
    r.p_wdv += G.poff;
  }
}

// k_reduce over the groups of one mode: wave -> group by a (scalar) binary
// search of the launch's wave offsets, then the single-group wave body.
template <int AGG, int MODE, bool RATE, bool DONLY>
__global__ void __launch_bounds__(256) k_reduce_seg(ReduceArgs r0, SegReduce s) {
  const uint64_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * blockDim.x + threadIdx.x) / WAVE);
  if (wave >= s.wv_start[s.n]) return;
  uint32_t lo = 0, hi = s.n;  // wv_start[lo] <= wave < wv_start[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (s.wv_start[mid] <= wave) lo = mid; else hi = mid;
  }
  const SegGroup G = s.sg[s.glist[lo]];
  ReduceArgs r = r0;
  seg_view(r, G);
  reduce_wave<AGG, MODE, RATE, DONLY>(r, (uint32_t)(wave - s.wv_start[lo]), nullptr);
}

// k_finalize_seq over every grid point of the groups of one mode.
template <int AGG, int MODE, bool RATE>
__global__ void __launch_bounds__(256) k_finalize_seg(ReduceArgs r0, FinalArgs f0, const SegGroup* sg,
                                                      const uint64_t* goff, uint32_t n_groups, uint64_t T_all,
                                                      GroupDev* gd) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= T_all) return;
  uint32_t lo = 0, hi = n_groups;  // last group with goff <= t (empty groups share the next offset)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (goff[mid] <= t) lo = mid; else hi = mid;
  }
  const SegGroup G = sg[lo];
  if (G.mode != (uint32_t)MODE || t - G.goff >= G.T) return;
  ReduceArgs r = r0;
  seg_view(r, G);
  FinalArgs f = f0;
  f.T = G.T;
  f.n_chunks = G.n_chunks;
  f.grid += G.goff;
  f.fstar = G.fstar;
  f.out_ts += G.goff;
  f.out_isint += G.goff;
  f.out_bits += G.goff;
  f.nan_t = &gd[lo].nan_t;
  const uint64_t g = t - G.goff;
  Acc a;
  acc_load<AGG, MODE>(r, g, a);
  for (uint32_t c = 1; c < f.n_chunks; c++) {
    Acc b;
    acc_load<AGG, MODE>(r, (uint64_t)c * f.T + g, b);
    acc_merge<AGG, MODE>(a, b);
  }
  finalize_one<AGG, MODE, RATE>(f, g, a);
}

// ---- the direct no-downsampling path per group (k_direct.hip) -------------
// Marks each direct candidate's points {x0 + i*step} in its group's bitmap:
// wave per 64 candidates, runs of the same (group, pattern) marked once.
__global__ void __launch_bounds__(256) k_direct_mark_seg(DirectArgs dg, uint32_t n_kept, const uint32_t* kgrp,
                                                         GroupGrid q, uint32_t* bitmap) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  uint32_t m_g = ~0u, m_step = 0, m_np = 0;
  int64_t m_xf = -1;
  for (uint32_t kb = ufl(wave) * WAVE; kb < n_kept; kb += nwaves * WAVE) {
    const uint32_t k = kb + lane;
    uint32_t info = 0, x0 = 0, step = 0, ne = 0, g = 0;
    if (k < n_kept) {
      info = dg.info[k];
      if (info & DIR_ON) {
        x0 = dg.x0[k];
        step = dg.step[k];
        ne = dg.n[k];
        g = kgrp[k];
      }
    }
    uint64_t todo = ballot((info & DIR_ON) != 0);
    while (todo) {
      const int j = __builtin_ctzll(todo);
      todo &= todo - 1;
      const uint32_t gj = readlane_u32(g, j), sj = readlane_u32(step, j), nj = readlane_u32(ne, j);
      const int64_t xj = (int64_t)readlane_u32(x0, j);
      const int64_t xf = dg.rate ? xj + sj : xj;
      const uint32_t np = dg.rate ? nj - 1 : nj;
      if (np == 0 || (gj == m_g && xf == m_xf && sj == m_step && np == m_np)) continue;
      DirectArgs v = dg;
      v.bitmap = bitmap + q.wbase[gj];
      v.lo = q.lo[gj];
      direct_mark(v, xf, sj, np);
      m_g = gj;
      m_xf = xf;
      m_step = sj;
      m_np = np;
    }
  }
}

// k_direct_verify against each candidate's group grid (word ranks rebased).
__global__ void __launch_bounds__(256) k_direct_verify_seg(DirectArgs dg, uint32_t n_kept, const uint32_t* kgrp,
                                                           GroupGrid q, const uint32_t* bitmap,
                                                           const uint32_t* word_rank) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  bool fail = false;
  if (k < n_kept) {
    const uint32_t info = dg.info[k];
    if (info & DIR_ON) {
      const uint32_t ne = dg.n[k], step = dg.step[k];
      const int64_t x0 = dg.x0[k];
      const int64_t xf = dg.rate ? x0 + step : x0;
      const uint32_t np = dg.rate ? ne - 1 : ne;
      if (np == 0) {
        dg.ga[k] = 0;
      } else {
        const uint32_t g = kgrp[k];
        const uint64_t wb = q.wbase[g];
        const int64_t xl = x0 + (int64_t)(ne - 1) * step;
        const uint32_t ra = grid_rank(bitmap + wb, word_rank + wb, q.lo[g], xf);
        const uint32_t rl = grid_rank(bitmap + wb, word_rank + wb, q.lo[g], xl);
        dg.ga[k] = ra;
        if (rl - ra != np - 1) {
          fail = true;
          dg.info[k] = 0;
        }
      }
    }
  }
  const uint64_t m = ballot(fail);
  if (m) {
    const int lane = lane_id();
    uint32_t base = 0;
    if (lane == __builtin_ctzll(m)) base = atomicAdd(dg.list_count, (uint32_t)__popcll(m));
    base = __shfl(base, __builtin_ctzll(m));
    if (fail) dg.list[base + __popcll(m & lanemask_lt(lane))] = k;
  }
}

// k_chunk_flags per group: chunk c of group g holds an E span.
__global__ void k_chunk_flags_seg(const uint32_t* d_info, uint32_t n_kept, const uint32_t* kgrp,
                                  const SegGroup* sg, const uint64_t* choff, uint32_t* chunk_e) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_kept || (d_info[k] & DIR_ON)) return;
  const uint32_t g = kgrp[k];
  const SegGroup G = sg[g];
  if (!G.T) return;
  chunk_e[choff[g] + (k - G.k0) / G.spc] = 1u;
}

}  // namespace tsdb
