// k_grid.hip — the SGIterator emission times G (SpanGroup.java:510-577):
// the sorted distinct timestamps of every span's next-slot points <= end,
// i.e. G = sorted-unique{ e.ts <= end } (rate: points e_j, j >= 1).
//
// G is built as a bitmap over [lo, hi] (hi = min(end, max E ts)): one bit per
// second, then a word-popcount prefix gives rank(t) = |{g in G : g < t}| in
// O(1), which the reducer uses to place span points on the grid. Bitmap size
// is (hi - lo + 1) / 8 bytes (<= 512 MiB for any u32 range; ~5 MB for the
// 40 M-second C4 range) and stays L2/MALL resident while marked.
#pragma once
#include "dev_common.h"

namespace tsdb {

struct GridArgs {
  const uint64_t* e_off;
  const uint32_t* e_len;
  const uint32_t* e_ts;
  uint32_t n_kept;
  int64_t lo, hi;       // bitmap covers [lo, hi]
  int32_t rate;
  uint32_t* bitmap;     // [nwords]
  uint64_t nwords;
  uint32_t* word_rank;  // [nwords] exclusive prefix of popcounts
  uint32_t* block_sum;  // [nblocks]
  uint32_t* grid;       // [T] G
  uint64_t* total;      // [1] T
  const uint32_t* list;       // k_grid_mark: only these kept spans (null: all)
  const uint32_t* list_count;
  uint32_t* zero2;            // k_grid_popc: two list counters to zero for the
                              // kernels after the grid (null: none)
  // k_grid_mark also does k_span_summary's work for its spans when err is set:
  // an empty E raises E_EMPTY_SPAN, a float first point raises F* (non-rate)
  const uint8_t* e_flt;
  unsigned long long* err;
  unsigned long long* fstar;
  HostPub pub;                // the call state to the host once T is known (the
  const uint64_t* pub_src;    // single-block kernel that writes T publishes it)
  // sharded calls: two independent 64-bit hashes of the bitmap words (word
  // value and index), summed over words, so ranks can tell whether their
  // local grids agree; null: not computed
  unsigned long long* hash;        // [2]
  unsigned long long* block_hash;  // [2 nblocks] (more than one block)
  // k_grid_popc over a single block (nwords <= 1024): also emits G here
  // (its ranks are final), one launch fewer (null: k_grid_emit / k_emit_verify do)
  uint32_t* emit1;
};

// the per-word terms of the two grid hashes (splitmix64 finalisers of the
// word and its index; a sum of them over all words)
DEVI uint64_t gh_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
DEVI uint64_t gh_term1(uint32_t word, uint64_t w) { return gh_mix(((uint64_t)word << 32 | (w & 0xFFFFFFFFull)) + 0x9E3779B97F4A7C15ull); }
DEVI uint64_t gh_term2(uint32_t word, uint64_t w) { return gh_mix((uint64_t)word * 0xD1B54A32D192ED03ull ^ (w * 0x8CB92BA72F3D8DD7ull + 1)); }

// Mark every candidate point. Many spans share timestamps (regular cadence),
// so test before the atomic: a word that already has the bit skips it.
__global__ void __launch_bounds__(256) k_grid_mark(GridArgs g) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  const uint32_t n = g.list ? *g.list_count : g.n_kept;
  int64_t fs = 0;  // F* + 1 of this wave's spans (0: none)
  bool empty = false;
  for (uint32_t w = wave; w < n; w += nwaves) {
    const uint32_t k = g.list ? g.list[w] : w;
    const uint64_t eo = g.e_off[k];
    const uint32_t len = g.e_len[k];
    if (g.err) {
      empty |= len == 0;
      if (len && !g.rate && g.e_flt[eo]) fs = max(fs, (int64_t)g.e_ts[eo] + 1);
    }
    for (uint32_t i0 = g.rate ? 1 : 0; i0 < len; i0 += WAVE) {
      const uint32_t i = i0 + lane;
      if (i >= len) break;
      const int64_t t = g.e_ts[eo + i];
      if (t > g.hi) break;  // sorted: the rest are beyond end
      if (t < g.lo) continue;
      const uint64_t b = (uint64_t)(t - g.lo);
      const uint32_t bit = 1u << (b & 31);
      uint32_t* w = &g.bitmap[b >> 5];
      if (!(*w & bit)) atomicOr(w, bit);
    }
  }
  if (g.err && lane == 0) {  // (wave-uniform values)
    if (empty) err_raise(g.err, 2, 0, -3 /*E_EMPTY_SPAN*/);
    if (fs && (unsigned long long)fs > *(volatile unsigned long long*)g.fstar)
      atomicMax(g.fstar, (unsigned long long)fs);
  }
}

// ---- the sliced grid marking (long grids of sparse spans, C4) ----
// k_grid_mark's one atomic a point lands on a random word of a bitmap far
// larger than an XCD's L2 (C4: 11.7M points over ~2.5M words: ~140 B of
// fabric traffic a point). Instead the bitmap is cut into slices of GM_WORDS
// words a block owns: k_grid_bounds records, for every marked span, the
// first E index of each slice (one pass over E, coalesced); k_grid_mark_slices
// then marks a slice in LDS from every span's points inside it and ORs the
// slice into the bitmap with plain stores (one read, one write a word).
constexpr uint32_t GM_SHIFT = 13, GM_WORDS = 1u << GM_SHIFT;  // 32 KB of LDS a slice

DEVI int64_t gm_slice(const GridArgs& g, int64_t t) { return (t - g.lo) >> (5 + GM_SHIFT); }

// wave per marked span w (k = list[w] or w): B[sl * nm + w] = the first of
// the span's marked points (E indices [i0, iend): i0 = 1 with rate, iend the
// first point past hi) in slice sl or later, iend if none, for sl in [0,
// n_sl]; also the empty-span / F* work of k_grid_mark
__global__ void __launch_bounds__(256) k_grid_bounds(GridArgs g, uint32_t* B, uint32_t n_sl) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  const uint32_t nm = g.list ? *g.list_count : g.n_kept;
  int64_t fs = 0;
  bool empty = false;
  for (uint32_t w = wave; w < nm; w += nwaves) {
    const uint32_t k = g.list ? g.list[w] : w;
    const uint64_t eo = g.e_off[k];
    const uint32_t len = g.e_len[k];
    if (g.err) {
      empty |= len == 0;
      if (len && !g.rate && g.e_flt[eo]) fs = max(fs, (int64_t)g.e_ts[eo] + 1);
    }
    const uint32_t i0 = g.rate ? 1u : 0u;
    uint32_t iend = max(len, i0);
    int64_t last_sl = -1;  // slice of the last marked point so far
    for (uint32_t b = i0; b < iend; b += WAVE) {
      const uint32_t i = b + lane;
      const bool valid = i < iend;
      const int64_t t = valid ? (int64_t)g.e_ts[eo + i] : 0;
      const uint64_t past = ballot(valid && t > g.hi);
      const uint32_t lim = past ? b + (uint32_t)__builtin_ctzll(past) : iend;
      const bool mine = i < lim;
      const int64_t sl = mine ? gm_slice(g, t) : 0;
      int64_t sp = (int64_t)shfl_up_u64((uint64_t)sl, 1);
      if (lane == 0) sp = last_sl;
      if (mine)
        for (int64_t s2 = sp + 1; s2 <= sl; s2++) B[(uint64_t)s2 * nm + w] = i;
      if (lim > b) last_sl = (int64_t)readlane_u64((uint64_t)sl, (int)min(lim - b, (uint32_t)WAVE) - 1);
      if (past) {
        iend = lim;
        break;
      }
    }
    for (int64_t sl = last_sl + 1 + lane; sl <= (int64_t)n_sl; sl += WAVE) B[(uint64_t)sl * nm + w] = iend;
  }
  if (g.err && lane == 0) {
    if (empty) err_raise(g.err, 2, 0, -3 /*E_EMPTY_SPAN*/);
    if (fs && (unsigned long long)fs > *(volatile unsigned long long*)g.fstar)
      atomicMax(g.fstar, (unsigned long long)fs);
  }
}

// block per slice: the marked spans' points inside it set in LDS, then OR-ed
// into the bitmap's words of the slice
__global__ void __launch_bounds__(256) k_grid_mark_slices(GridArgs g, const uint32_t* B, uint32_t n_sl) {
  __shared__ uint32_t s_w[GM_WORDS];
  const uint32_t sl = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < GM_WORDS; i += 256) s_w[i] = 0;
  __syncthreads();
  const uint32_t nm = g.list ? *g.list_count : g.n_kept;
  const int lane = lane_id();
  const uint64_t wbase = (uint64_t)sl << GM_SHIFT;
  for (uint32_t w = threadIdx.x / WAVE; w < nm; w += 4) {
    const uint32_t k = g.list ? g.list[w] : w;
    const uint32_t a = B[(uint64_t)sl * nm + w], b = B[(uint64_t)(sl + 1) * nm + w];
    if (a >= b) continue;
    const uint64_t eo = g.e_off[k];
    for (uint32_t i = a + lane; i < b; i += WAVE) {
      const uint64_t bit = (uint64_t)((int64_t)g.e_ts[eo + i] - g.lo);
      atomicOr(&s_w[(bit >> 5) - wbase], 1u << (bit & 31));
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < GM_WORDS; i += 256) {
    const uint64_t wd = wbase + i;
    if (wd < g.nwords && s_w[i]) g.bitmap[wd] |= s_w[i];
  }
}

// Per-block (1024 words) exclusive popcount prefix.
__global__ void __launch_bounds__(256) k_grid_popc(GridArgs g) {
  __shared__ uint32_t s_wave[4];
  __shared__ unsigned long long s_h[2][4];
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
  const int t = threadIdx.x;
  uint32_t c[4];
  uint32_t tot = 0;
  uint64_t h1 = 0, h2 = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t w = base + t * 4 + i;
    const uint32_t word = w < g.nwords ? g.bitmap[w] : 0u;
    c[i] = __popc(word);
    tot += c[i];
    if (g.hash && w < g.nwords) {
      h1 += gh_term1(word, w);
      h2 += gh_term2(word, w);
    }
  }
  if (g.hash) {  // (block sums of the two hashes)
    for (int o = 1; o < WAVE; o <<= 1) {
      h1 += shfl_xor_u64(h1, o);
      h2 += shfl_xor_u64(h2, o);
    }
    if ((t & 63) == 0) {
      s_h[0][t >> 6] = h1;
      s_h[1][t >> 6] = h2;
    }
  }
  const uint32_t incl = wave_incl_scan_u32(tot);
  if ((t & 63) == 63) s_wave[t >> 6] = incl;
  __syncthreads();
  uint32_t woff = 0;
  for (int i = 0; i < (t >> 6); i++) woff += s_wave[i];
  uint32_t run = woff + incl - tot;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t w = base + t * 4 + i;
    if (w < g.nwords) {
      g.word_rank[w] = run;
      if (g.emit1 && gridDim.x == 1) {  // (one block: run is the final rank)
        uint32_t bits = g.bitmap[w], j = run;
        while (bits) {
          g.emit1[j++] = (uint32_t)(g.lo + (int64_t)(w * 32 + __builtin_ctz(bits)));
          bits &= bits - 1;
        }
      }
    }
    run += c[i];
  }
  if (t == 0 && blockIdx.x == 0 && g.zero2) {  // (their last readers ran before this kernel)
    g.zero2[0] = 0;
    g.zero2[1] = 0;
  }
  if (t == 255) {
    g.block_sum[blockIdx.x] = woff + incl;
    if (g.hash) {  // (s_h is complete: the __syncthreads above)
      const uint64_t b1 = s_h[0][0] + s_h[0][1] + s_h[0][2] + s_h[0][3];
      const uint64_t b2 = s_h[1][0] + s_h[1][1] + s_h[1][2] + s_h[1][3];
      if (gridDim.x == 1) {
        g.hash[0] = b1 | 1ull;  // (never 0: 0 stands for an empty grid)
        g.hash[1] = b2;
      } else {
        g.block_hash[2 * blockIdx.x] = b1;
        g.block_hash[2 * blockIdx.x + 1] = b2;
      }
    }
    if (gridDim.x == 1) {  // one block: its offset is 0 and its sum is T (no k_grid_scan_blocks)
      g.block_sum[0] = 0;
      g.total[0] = woff + incl;
      __threadfence();
    }
  }
  if (gridDim.x == 1 && g.pub.dst && t >= 192) {  // (the wave holding thread 255)
    __builtin_amdgcn_wave_barrier();
    host_publish(g.pub, g.pub_src);
  }
}

// Single block: exclusive scan of the block sums; writes T.
__global__ void __launch_bounds__(256) k_grid_scan_blocks(GridArgs g, uint32_t nblocks) {
  __shared__ uint32_t s_wave[4];
  __shared__ uint32_t s_carry;
  const int t = threadIdx.x;
  if (t == 0) s_carry = 0;
  __syncthreads();
  for (uint32_t b0 = 0; b0 < nblocks; b0 += 256) {
    const uint32_t b = b0 + t;
    const uint32_t v = b < nblocks ? g.block_sum[b] : 0;
    const uint32_t incl = wave_incl_scan_u32(v);
    if ((t & 63) == 63) s_wave[t >> 6] = incl;
    __syncthreads();
    uint32_t woff = 0;
    for (int i = 0; i < (t >> 6); i++) woff += s_wave[i];
    const uint32_t carry = s_carry;
    if (b < nblocks) g.block_sum[b] = carry + woff + incl - v;
    __syncthreads();
    if (t == 255) s_carry = carry + woff + incl;
    __syncthreads();
  }
  if (g.hash && t < WAVE) {  // the block hashes summed (wrapping), wave 0
    uint64_t h1 = 0, h2 = 0;
    for (uint32_t b = t; b < nblocks; b += WAVE) {
      h1 += g.block_hash[2 * b];
      h2 += g.block_hash[2 * b + 1];
    }
    for (int o = 1; o < WAVE; o <<= 1) {
      h1 += shfl_xor_u64(h1, o);
      h2 += shfl_xor_u64(h2, o);
    }
    if (t == 0) {
      g.hash[0] = h1 | 1ull;
      g.hash[1] = h2;
    }
  }
  if (t == 0) {
    g.total[0] = s_carry;
    __threadfence();
  }
  if (g.pub.dst && t < WAVE) {
    __builtin_amdgcn_wave_barrier();
    host_publish(g.pub, g.pub_src);
  }
}

// Adds block offsets and materializes G.
__global__ void __launch_bounds__(256) k_grid_emit(GridArgs g) {
  const uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (w >= g.nwords) return;
  const uint32_t r = g.word_rank[w] + g.block_sum[w >> 10];
  g.word_rank[w] = r;
  uint32_t bits = g.bitmap[w];
  uint32_t i = r;
  while (bits) {
    const int b = __builtin_ctz(bits);
    g.grid[i++] = (uint32_t)(g.lo + (int64_t)(w * 32 + b));
    bits &= bits - 1;
  }
}

// k_grid_emit that leaves the block-local ranks in place and writes the final
// ones to rank_out, so a kernel fused beside it (k_emit_verify) can read them.
DEVI void grid_emit_to(const GridArgs& g, uint64_t w, uint32_t* rank_out) {
  if (w >= g.nwords) return;
  const uint32_t r = g.word_rank[w] + g.block_sum[w >> 10];
  rank_out[w] = r;
  uint32_t bits = g.bitmap[w];
  uint32_t i = r;
  while (bits) {
    const int b = __builtin_ctz(bits);
    g.grid[i++] = (uint32_t)(g.lo + (int64_t)(w * 32 + b));
    bits &= bits - 1;
  }
}

// rank(t): number of grid points < t (t must lie in [lo, hi+1)).
DEVI uint32_t grid_rank(const uint32_t* bitmap, const uint32_t* word_rank, int64_t lo, int64_t t) {
  const uint64_t b = (uint64_t)(t - lo);
  const uint64_t w = b >> 5;
  return word_rank[w] + __popc(bitmap[w] & ((1u << (b & 31)) - 1));
}

// the same from the block-local ranks and the block offsets (before k_grid_emit)
DEVI uint32_t grid_rank2(const uint32_t* bitmap, const uint32_t* word_rank, const uint32_t* block_sum, int64_t lo,
                         int64_t t) {
  const uint64_t b = (uint64_t)(t - lo);
  const uint64_t w = b >> 5;
  return word_rank[w] + block_sum[w >> 10] + __popc(bitmap[w] & ((1u << (b & 31)) - 1));
}

// End of a single-group call (api.hip), after the finalize: every set bit of
// the bitmap is a grid point, so clearing the word of each grid point leaves
// the whole bitmap zero for the next call (no memset per call).
__global__ void __launch_bounds__(256) k_bitmap_clear(uint32_t* bitmap, const uint32_t* grid, uint64_t T, int64_t lo) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < T; i += (uint64_t)gridDim.x * 256)
    bitmap[(uint64_t)((int64_t)grid[i] - lo) >> 5] = 0u;
}

}  // namespace tsdb
