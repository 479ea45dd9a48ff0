// k_util.hip — device-wide exclusive scan (u64), kept-span compaction, the
// synthetic KeyValue generator, and the lazy-error index.
#pragma once
#include "dev_common.h"
#include "k_grid.hip"

namespace tsdb {

// ---- exclusive scan over u64 (1024 elements per block) --------------------
__global__ void __launch_bounds__(256) k_scan_block_u64(const uint64_t* in, uint64_t* out, uint64_t n,
                                                        uint64_t* block_sums) {
  __shared__ uint64_t s_wave[4];
  const uint64_t base = (uint64_t)blockIdx.x * 1024;
  const int t = threadIdx.x;
  uint64_t v[4];
  uint64_t tot = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t e = base + t * 4 + i;
    v[i] = e < n ? in[e] : 0;
    tot += v[i];
  }
  const uint64_t incl = wave_incl_scan_u64(tot);
  if ((t & 63) == 63) s_wave[t >> 6] = incl;
  __syncthreads();
  uint64_t woff = 0;
  for (int i = 0; i < (t >> 6); i++) woff += s_wave[i];
  uint64_t run = woff + incl - tot;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t e = base + t * 4 + i;
    if (e < n) out[e] = run;
    run += v[i];
  }
  if (t == 255) block_sums[blockIdx.x] = woff + incl;
}

__global__ void __launch_bounds__(256) k_scan_blocks_u64(uint64_t* block_sums, uint64_t nb, uint64_t* total) {
  __shared__ uint64_t s_wave[4];
  __shared__ uint64_t s_carry;
  const int t = threadIdx.x;
  if (t == 0) s_carry = 0;
  __syncthreads();
  for (uint64_t b0 = 0; b0 < nb; b0 += 256) {
    const uint64_t b = b0 + t;
    const uint64_t v = b < nb ? block_sums[b] : 0;
    const uint64_t incl = wave_incl_scan_u64(v);
    if ((t & 63) == 63) s_wave[t >> 6] = incl;
    __syncthreads();
    uint64_t woff = 0;
    for (int i = 0; i < (t >> 6); i++) woff += s_wave[i];
    const uint64_t carry = s_carry;
    if (b < nb) block_sums[b] = carry + woff + incl - v;
    __syncthreads();
    if (t == 255) s_carry = carry + woff + incl;
    __syncthreads();
  }
  if (t == 0) *total = s_carry;
}

__global__ void __launch_bounds__(256) k_scan_add_u64(uint64_t* out, uint64_t n, const uint64_t* block_sums) {
  const uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n) out[e] += block_sums[e >> 10];
}

// ---- kept spans ------------------------------------------------------------
__global__ void k_kept_flags(const uint8_t* kept, uint64_t* kflag, uint32_t n) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s < n) kflag[s] = kept[s];
}
// Kept-span list, E offsets, and (one atomic per block, grid-stride)
// SpanGroup.aggregatedSize and the [min first, max last] ts bounds of the
// kept spans.
__global__ void __launch_bounds__(256) k_kept_scatter(const uint8_t* kept, const uint64_t* kidx,
                                                      const uint64_t* eoff_s, const uint32_t* ncells, uint32_t n,
                                                      uint32_t* kept_list, uint64_t* eoff_k,
                                                      unsigned long long* n_input, const int64_t* sp_first,
                                                      const int64_t* sp_last, unsigned long long* bound) {
  __shared__ uint64_t sh_c[4];
  __shared__ int64_t sh_f[4], sh_l[4];
  uint64_t cnt = 0;
  int64_t f = INT64_MAX, l = INT64_MIN;
  for (uint32_t s = blockIdx.x * blockDim.x + threadIdx.x; s < n; s += gridDim.x * blockDim.x) {
    if (!kept[s]) continue;
    const uint64_t k = kidx[s];
    kept_list[k] = s;
    eoff_k[k] = eoff_s[s];
    cnt += ncells[s];
    f = min(f, sp_first[s]);
    l = max(l, sp_last[s]);
  }
  cnt = block_reduce_256(cnt, [](uint64_t x, uint64_t y) { return x + y; }, sh_c);
  f = block_reduce_256(f, [](int64_t x, int64_t y) { return min(x, y); }, sh_f);
  l = block_reduce_256(l, [](int64_t x, int64_t y) { return max(x, y); }, sh_l);
  if (threadIdx.x == 0 && cnt) {
    atomicAdd(n_input, (unsigned long long)cnt);
    atomicMin(&bound[0], (unsigned long long)f);
    atomicMax(&bound[1], (unsigned long long)l);
  }
}

// The same in one launch for groups of up to KC_MAX spans (replaces
// k_kept_flags + two 3-kernel scans + k_kept_scatter): one 1024-thread block
// walks the spans 4096 at a time, carrying the two running prefixes. (A
// multi-block single pass would need a look-back across the XCDs' separate
// L2s, i.e. device-scope fences per tile: slower than the scan kernels.)
#ifndef KC_MAX_LOG2
#define KC_MAX_LOG2 12  // (14: C2 0.391 ms device step, 12: 0.381 — the 10k-span single block took 22 us)
#endif
constexpr uint32_t KC_MAX = 1u << KC_MAX_LOG2;
struct KeptArgs {
  const uint8_t* kept;
  const uint64_t* cap;
  const uint32_t* ncells;
  uint32_t n;
  uint32_t* kept_list;
  uint64_t* eoff_k;
  unsigned long long* n_input;
  const int64_t* sp_first;
  const int64_t* sp_last;
  unsigned long long* bound;
  uint64_t* n_kept_out;
  uint64_t* e_total_out;
  HostPub pub;
  const uint64_t* pub_src;
  // the uniform-group proposal (null: not made): the spans' keys and row
  // offsets (AssembleArgs.u_*), the kept spans' offsets by kept index, and
  // the keys' [min, max, min, max] over the kept spans (Small.ukey)
  const uint64_t* u_key1;
  const uint64_t* u_key2;
  const uint64_t* u_vo;
  const uint64_t* u_qo;
  uint64_t* uk_vo;
  uint64_t* uk_qo;
  unsigned long long* ukey;
  // (null: not wanted) the speculative aligned group's verdict, written with
  // the keys: ug_spec_fits(keys, n_kept, *err, ug_interval)
  uint32_t* ug_go;
  const unsigned long long* err;
  int64_t ug_interval;
};
// [min, max] of the kept spans' keys (uniform-group proposal), per thread
struct UKeyAcc {
  uint64_t a0, a1, b0, b1;
  DEVI void init() { a0 = b0 = ~0ull; a1 = b1 = 0; }
  DEVI void add(uint64_t k1, uint64_t k2) {
    a0 = min(a0, k1); a1 = max(a1, k1); b0 = min(b0, k2); b1 = max(b1, k2);
  }
  DEVI void add(const UKeyAcc& o) {
    a0 = min(a0, o.a0); a1 = max(a1, o.a1); b0 = min(b0, o.b0); b1 = max(b1, o.b1);
  }
  DEVI void wave_reduce() {
#pragma unroll
    for (int m = 1; m < WAVE; m <<= 1) {
      a0 = min(a0, shfl_xor_u64(a0, m)); a1 = max(a1, shfl_xor_u64(a1, m));
      b0 = min(b0, shfl_xor_u64(b0, m)); b1 = max(b1, shfl_xor_u64(b1, m));
    }
  }
};
// (a 1024-thread block)
DEVI void kept_compact_block(const KeptArgs& A) {
  const uint8_t* kept = A.kept; const uint64_t* cap = A.cap; const uint32_t* ncells = A.ncells;
  const uint32_t n = A.n; uint32_t* kept_list = A.kept_list; uint64_t* eoff_k = A.eoff_k;
  unsigned long long* n_input = A.n_input; const int64_t* sp_first = A.sp_first; const int64_t* sp_last = A.sp_last;
  unsigned long long* bound = A.bound; uint64_t* n_kept_out = A.n_kept_out; uint64_t* e_total_out = A.e_total_out;
  const HostPub& pub = A.pub; const uint64_t* pub_src = A.pub_src;
  __shared__ uint64_t s_wk[16], s_we[16];
  __shared__ uint64_t s_c[16];
  __shared__ int64_t s_f[16], s_l[16], s_fx[16], s_ln[16];
  __shared__ UKeyAcc s_u[16];
  UKeyAcc u;
  u.init();
  const int t = threadIdx.x, lane = lane_id(), w = t / WAVE;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  uint64_t ck = 0, ce = 0;  // carries: kept spans / E capacity before this round
  uint64_t cnt = 0;
  int64_t f = INT64_MAX, l = INT64_MIN, fx = INT64_MIN, ln = INT64_MAX;
  for (uint64_t base0 = 0; base0 < n; base0 += 4096) {
    const uint64_t base = base0 + 4 * t;
    uint32_t fk[4], fn[4];
    uint64_t fe[4], sk = 0, se = 0;
    int64_t ff[4], fl[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {  // (branch-free: every load of the round in flight together)
      const uint64_t s = base + i;
      const bool in = s < n;
      const uint64_t sc = in ? s : n - 1;
      const uint32_t kb = kept[sc];
      const uint64_t cb = cap[sc];
      fn[i] = ncells[sc];
      ff[i] = sp_first[sc];
      fl[i] = sp_last[sc];
      fk[i] = in && kb ? 1u : 0u;
      fe[i] = in ? cb : 0ull;
      sk += fk[i];
      se += fe[i];
    }
    const uint64_t ik = wave_incl_scan_u64_dpp(sk), ie = wave_incl_scan_u64_dpp(se);
    if (lane == 63) {
      s_wk[w] = ik;
      s_we[w] = ie;
    }
    __syncthreads();
    // the 16 wave sums scanned across lanes (not 32 LDS loads per thread)
    const uint64_t pk = wave_incl_scan_u64_dpp(lane < 16 ? s_wk[lane] : 0ull);
    const uint64_t pe = wave_incl_scan_u64_dpp(lane < 16 ? s_we[lane] : 0ull);
    const uint64_t wk = wu ? readlane_u64(pk, wu - 1) : 0ull, we = wu ? readlane_u64(pe, wu - 1) : 0ull;
    const uint64_t tk = readlane_u64(pk, 15), te = readlane_u64(pe, 15);
    __syncthreads();  // (s_wk reused next round)
    uint64_t rk = ck + wk + ik - sk, re = ce + we + ie - se;
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint64_t s = base + i;
      if (fk[i]) {
        kept_list[rk] = (uint32_t)s;
        eoff_k[rk] = re;
        if (A.u_key1) {
          u.add(A.u_key1[s], A.u_key2[s]);
          A.uk_vo[rk] = A.u_vo[s];
          A.uk_qo[rk] = A.u_qo[s];
        }
        cnt += fn[i];
        f = min(f, ff[i]);
        l = max(l, fl[i]);
        fx = max(fx, ff[i]);
        ln = min(ln, fl[i]);
      }
      rk += fk[i];
      re += fe[i];
    }
    ck += tk;
    ce += te;
  }
  // block totals: aggregatedSize and the kept spans' [min first, max last]
#pragma unroll
  for (int m = 1; m < WAVE; m <<= 1) {
    cnt += shfl_xor_u64(cnt, m);
    f = min(f, (int64_t)shfl_xor_u64((uint64_t)f, m));
    l = max(l, (int64_t)shfl_xor_u64((uint64_t)l, m));
    fx = max(fx, (int64_t)shfl_xor_u64((uint64_t)fx, m));
    ln = min(ln, (int64_t)shfl_xor_u64((uint64_t)ln, m));
  }
  if (A.u_key1) u.wave_reduce();
  if (lane == 0) {
    s_c[w] = cnt;
    s_f[w] = f;
    s_l[w] = l;
    s_fx[w] = fx;
    s_ln[w] = ln;
    s_u[w] = u;
  }
  __syncthreads();
  if (t == 0) {
    for (int i = 1; i < 16; i++) {
      cnt += s_c[i];
      f = min(f, s_f[i]);
      l = max(l, s_l[i]);
      fx = max(fx, s_fx[i]);
      ln = min(ln, s_ln[i]);
      u.add(s_u[i]);
    }
    if (A.u_key1) {  // (the call state's initial keys are neutral: [~0, 0, ~0, 0])
      A.ukey[0] = min((uint64_t)A.ukey[0], u.a0); A.ukey[1] = max((uint64_t)A.ukey[1], u.a1);
      A.ukey[2] = min((uint64_t)A.ukey[2], u.b0); A.ukey[3] = max((uint64_t)A.ukey[3], u.b1);
    }
    *n_kept_out = ck;
    *e_total_out = ce;
    if (A.ug_go)
      *A.ug_go = ug_spec_fits(A.ukey[0], A.ukey[1], A.ukey[2], A.ukey[3], ck, *A.err, A.ug_interval) ? 1u : 0u;
    if (cnt) {
      atomicAdd(n_input, (unsigned long long)cnt);
      atomicMin(&bound[0], (unsigned long long)f);
      atomicMax(&bound[1], (unsigned long long)l);
      atomicMax(&bound[2], (unsigned long long)fx);
      atomicMin(&bound[3], (unsigned long long)ln);
    }
  }
  if (pub.dst && t < WAVE) {  // the call state, final here, to the host (wave 0)
    __threadfence();
    __builtin_amdgcn_wave_barrier();
    host_publish(pub, pub_src);
  }
}
__global__ void __launch_bounds__(1024) k_kept_compact(KeptArgs A) { kept_compact_block(A); }

// Bigger groups in two launches: per tile of 1024 spans its sums (kept,
// capacity, cells) and bounds; then each tile adds up its predecessors' sums
// itself (at most a few thousand tiles: no serial chain across tiles) and
// scatters, and the last tile's block, which reads every tile's sums anyway,
// writes the group's totals and bounds (no atomics from every block) and
// hands the call state to the host (no k_publish launch).
struct KeptTile {
  uint64_t k, e, cnt;
  int64_t f, l, fx, ln;  // over the tile's kept spans with cells (neutral otherwise)
  uint64_t pad;
  UKeyAcc u;             // the uniform-group keys over the tile's kept spans
};
// the block's UKeyAcc (256 threads) into thread 0's
DEVI UKeyAcc ukey_block_256(UKeyAcc u, UKeyAcc* sh /* [4] */) {
  u.wave_reduce();
  __syncthreads();
  if (lane_id() == 0) sh[threadIdx.x / WAVE] = u;
  __syncthreads();
  if (threadIdx.x == 0) {
    u.add(sh[1]);
    u.add(sh[2]);
    u.add(sh[3]);
  }
  return u;
}
__global__ void __launch_bounds__(256) k_kept_tiles(const uint8_t* kept, const uint64_t* cap, const uint32_t* ncells,
                                                    const int64_t* sp_first, const int64_t* sp_last, uint32_t n,
                                                    KeptTile* tile_sum, ulonglong2* tile_ke, const uint64_t* u_key1,
                                                    const uint64_t* u_key2) {
  __shared__ uint64_t sh_k[4], sh_e[4], sh_c[4];
  __shared__ int64_t sh_f[4], sh_l[4];
  __shared__ UKeyAcc sh_u[4];
  const uint64_t base = (uint64_t)blockIdx.x * 1024 + 4 * threadIdx.x;
  uint64_t sk = 0, se = 0, cnt = 0;
  int64_t f = INT64_MAX, l = INT64_MIN, fx = INT64_MIN, ln = INT64_MAX;
  UKeyAcc u;
  u.init();
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t s = base + i;
    if (s < n) {
      se += cap[s];
      if (kept[s]) {
        sk++;
        if (u_key1) u.add(u_key1[s], u_key2[s]);
        cnt += ncells[s];
        f = min(f, sp_first[s]);
        l = max(l, sp_last[s]);
        fx = max(fx, sp_first[s]);
        ln = min(ln, sp_last[s]);
      }
    }
  }
  sk = block_reduce_256(sk, [](uint64_t x, uint64_t y) { return x + y; }, sh_k);
  se = block_reduce_256(se, [](uint64_t x, uint64_t y) { return x + y; }, sh_e);
  cnt = block_reduce_256(cnt, [](uint64_t x, uint64_t y) { return x + y; }, sh_c);
  f = block_reduce_256(f, [](int64_t x, int64_t y) { return min(x, y); }, sh_f);
  l = block_reduce_256(l, [](int64_t x, int64_t y) { return max(x, y); }, sh_l);
  __syncthreads();
  fx = block_reduce_256(fx, [](int64_t x, int64_t y) { return max(x, y); }, sh_f);
  ln = block_reduce_256(ln, [](int64_t x, int64_t y) { return min(x, y); }, sh_l);
  if (u_key1) u = ukey_block_256(u, sh_u);
  if (threadIdx.x == 0) {
    KeptTile o;
    o.k = sk; o.e = se; o.cnt = cnt; o.pad = 0;
    o.u = u;
    // (a tile whose kept spans hold no cell leaves the bounds alone, as the
    // per-block atomics of the single-block path do)
    o.f = cnt ? f : INT64_MAX; o.l = cnt ? l : INT64_MIN; o.fx = cnt ? fx : INT64_MIN; o.ln = cnt ? ln : INT64_MAX;
    tile_sum[blockIdx.x] = o;
    tile_ke[blockIdx.x] = make_ulonglong2(sk, se);
  }
}

// (tile_ke: the kept / capacity sums of the producer's tiles, `sub` of them
// per 1024 spans of this kernel's tile, nt_sub in all: the prefix reads 16 B
// a producer tile, the last block every tile's whole sums)
__global__ void __launch_bounds__(256) k_kept_scatter_tiles(const uint8_t* kept, const uint64_t* cap, uint32_t n,
                                                            const KeptTile* tile_sum, const ulonglong2* tile_ke,
                                                            uint32_t sub, uint32_t nt_sub, uint32_t* kept_list,
                                                            uint64_t* eoff_k, unsigned long long* n_input,
                                                            unsigned long long* bound, uint64_t* n_kept_out,
                                                            uint64_t* e_total_out, HostPub pub,
                                                            const uint64_t* pub_src, KeptArgs U) {
  __shared__ uint64_t s_wk[4], s_we[4];
  __shared__ uint64_t sh_c[4];
  __shared__ int64_t sh_f[4], sh_l[4];
  __shared__ UKeyAcc sh_u[4];
  __shared__ uint64_t s_pk, s_pe;
  UKeyAcc u;
  u.init();
  const int t = threadIdx.x, lane = lane_id(), w = t / WAVE;
  const uint32_t tile = blockIdx.x;
  const bool last = tile == gridDim.x - 1;
  // this tile's offset: the sum of its predecessors' sums (the last tile: and
  // the totals of every tile)
  uint64_t pk = 0, pe = 0, cnt = 0;
  int64_t f = INT64_MAX, l = INT64_MIN, fx = INT64_MIN, ln = INT64_MAX;
  for (uint32_t q = t; q < tile * sub; q += 256) {
    const ulonglong2 v = tile_ke[q];
    pk += v.x;
    pe += v.y;
  }
  if (last)
    for (uint32_t q = t; q < nt_sub; q += 256) {
      const KeptTile v = tile_sum[q];
      cnt += v.cnt;
      f = min(f, v.f);
      l = max(l, v.l);
      fx = max(fx, v.fx);
      ln = min(ln, v.ln);
      u.add(v.u);
    }
  pk = block_reduce_256(pk, [](uint64_t x, uint64_t y) { return x + y; }, sh_c);
  __syncthreads();
  pe = block_reduce_256(pe, [](uint64_t x, uint64_t y) { return x + y; }, sh_c);
  if (t == 0) {
    s_pk = pk;
    s_pe = pe;
  }
  const uint64_t base = (uint64_t)tile * 1024 + 4 * t;
  uint32_t fk[4];
  uint64_t fe[4], sk = 0, se = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t s = base + i;
    fk[i] = s < n && kept[s] ? 1u : 0u;
    fe[i] = s < n ? cap[s] : 0ull;
    sk += fk[i];
    se += fe[i];
  }
  const uint64_t ik = wave_incl_scan_u64_dpp(sk), ie = wave_incl_scan_u64_dpp(se);
  if (lane == 63) {
    s_wk[w] = ik;
    s_we[w] = ie;
  }
  __syncthreads();
  uint64_t rk = s_pk + ik - sk, re = s_pe + ie - se;
  for (int i = 0; i < w; i++) {
    rk += s_wk[i];
    re += s_we[i];
  }
  if (t == 255 && last) {  // the totals
    *n_kept_out = rk + sk;
    *e_total_out = re + se;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint64_t s = base + i;
    if (fk[i]) {
      kept_list[rk] = (uint32_t)s;
      eoff_k[rk] = re;
      if (U.u_key1) {
        U.uk_vo[rk] = U.u_vo[s];
        U.uk_qo[rk] = U.u_qo[s];
      }
    }
    rk += fk[i];
    re += fe[i];
  }
  if (!last) return;
  __syncthreads();
  cnt = block_reduce_256(cnt, [](uint64_t x, uint64_t y) { return x + y; }, sh_c);
  f = block_reduce_256(f, [](int64_t x, int64_t y) { return min(x, y); }, sh_f);
  l = block_reduce_256(l, [](int64_t x, int64_t y) { return max(x, y); }, sh_l);
  __syncthreads();
  fx = block_reduce_256(fx, [](int64_t x, int64_t y) { return max(x, y); }, sh_f);
  __syncthreads();
  ln = block_reduce_256(ln, [](int64_t x, int64_t y) { return min(x, y); }, sh_l);
  if (U.u_key1) u = ukey_block_256(u, sh_u);
  if (t == 0 && U.u_key1) {
    U.ukey[0] = min((uint64_t)U.ukey[0], u.a0); U.ukey[1] = max((uint64_t)U.ukey[1], u.a1);
    U.ukey[2] = min((uint64_t)U.ukey[2], u.b0); U.ukey[3] = max((uint64_t)U.ukey[3], u.b1);
    if (U.ug_go)  // (n_kept_out: thread 255 of this block, before the reductions' barriers)
      *U.ug_go = ug_spec_fits(U.ukey[0], U.ukey[1], U.ukey[2], U.ukey[3], *n_kept_out, *U.err, U.ug_interval)
                     ? 1u : 0u;
  }
  if (t == 0 && cnt) {
    *n_input += cnt;
    bound[0] = min(bound[0], (unsigned long long)f);
    bound[1] = max(bound[1], (unsigned long long)l);
    bound[2] = max(bound[2], (unsigned long long)fx);
    bound[3] = min(bound[3], (unsigned long long)ln);
  }
  __syncthreads();
  if (pub.dst && t < WAVE) {  // the call state, final here, to the host (wave 0)
    __threadfence();
    __builtin_amdgcn_wave_barrier();
    host_publish(pub, pub_src);
  }
}

// ---- lazy error index (where the reference would throw) ----------------------
// A bad cell in E point k is read when point k-1 moves into the current slot
// (SpanGroup.java:583-608), i.e. while emitting ts(e_{k-1}); points 0 (and 1
// for rate) are read by the SGIterator constructor.
struct BadArgs {
  const int64_t* e_bad;
  const uint64_t* e_off;
  const uint32_t* e_ts;
  uint32_t n_kept;
  int32_t rate;
  int64_t hi, lo;
  const uint32_t* bitmap;
  const uint32_t* word_rank;
  uint64_t T;
};
// kept span k's error key (grid rank << 4 | code), ~0: none
DEVI uint64_t bad_key(const BadArgs& b, uint32_t k) {
  const int64_t e = b.e_bad[k];
  if (e < 0) return ~0ull;
  const uint64_t idx = (uint64_t)(e >> 4), code = (uint64_t)(e & 15);
  uint64_t at;
  if (idx == 0 || (b.rate && idx == 1)) {
    at = 0;
  } else {
    const int64_t tp = b.e_ts[b.e_off[k] + idx - 1];
    if (tp > b.hi) return ~0ull;  // never consumed
    at = b.T == 0 ? 0 : grid_rank(b.bitmap, b.word_rank, b.lo, tp);
  }
  return (at << 4) | code;
}
__global__ void k_bad_index(BadArgs b, unsigned long long* out) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= b.n_kept) return;
  const uint64_t key = bad_key(b, k);
  if (key != ~0ull) atomicMin(out, (unsigned long long)key);
}

// ---- synthetic KeyValues (bit-identical to opentsdb_amd/synth.py) -----------
DEVI uint64_t splitmix64(uint64_t x) {
  uint64_t z = x + 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
DEVI uint64_t hash3(uint64_t seed, uint64_t s, uint64_t i) {
  return splitmix64(splitmix64(seed ^ (s * 0xD1B54A32D192ED03ull)) ^ i);
}

struct SynthArgs {
  uint64_t seed;
  uint32_t n_spans, n_points, t0, step, kind, span0;
  uint32_t k;            // cells per full row
  uint32_t rps;          // rows per span
  uint32_t w;            // value width
  uint32_t flags;
  uint64_t qstride, vstride;
  uint64_t* span_row_start;
  uint32_t* row_base;
  uint32_t* row_ncells;
  uint64_t* row_qual_off;
  uint64_t* row_val_off;
  uint32_t* row_val_len;
  uint8_t* qual;
  uint8_t* val;
};

__global__ void k_synth_rows(SynthArgs a) {
  const uint64_t R = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t n_rows = (uint64_t)a.n_spans * a.rps;
  if (R == 0) a.span_row_start[a.n_spans] = n_rows;
  if (R >= n_rows) return;
  const uint64_t r = R % a.rps, s = R / a.rps;
  if (r == 0) a.span_row_start[s] = R;
  const int64_t left = (int64_t)a.n_points - (int64_t)r * a.k;
  const uint32_t nc = (uint32_t)(left < (int64_t)a.k ? left : a.k);
  a.row_ncells[R] = nc;
  a.row_base[R] = a.t0 + (uint32_t)r * 3600u;
  a.row_qual_off[R] = R * a.qstride;
  a.row_val_off[R] = R * a.vstride;
  a.row_val_len[R] = nc > 1 ? nc * a.w + 1 : nc * a.w;
}

__global__ void k_synth_cells(SynthArgs a) {
  const uint64_t cell = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t total = (uint64_t)a.n_spans * a.n_points;
  if (cell >= total) return;
  const uint64_t ls = cell / a.n_points, i = cell % a.n_points;
  const uint64_t row = ls * a.rps + i / a.k, c = i % a.k;
  const uint64_t s = ls + a.span0;  // global series index keys the hash
  const uint32_t q = (uint32_t)((c * a.step) << 4) | a.flags;
  uint8_t* qp = a.qual + row * a.qstride + 2 * c;
  qp[0] = (uint8_t)(q >> 8);
  qp[1] = (uint8_t)q;
  uint64_t be;  // value bytes, big-endian, in the low a.w bytes
  if (a.kind == 0) {
    const uint64_t base = hash3(a.seed, s, 0xFFFFFFFFull) >> 24;
    const uint64_t rr = hash3(a.seed, s, i) % 500ull;
    be = base + 500ull * i + rr;
  } else {
    const uint64_t h = hash3(a.seed, s, i);
    const int64_t sum = (int64_t)((h & 0xFFFF) + ((h >> 16) & 0xFFFF) + ((h >> 32) & 0xFFFF) + ((h >> 48) & 0xFFFF)) - 131070;
    const double prod = (double)sum * 0x1.bb685d0b4e463p-16;  // 1/37837
    const double v = 100.0 + prod;
    if (a.kind == 1) be = (uint64_t)__float_as_uint((float)v);
    else be = (uint64_t)__double_as_longlong(v);
  }
  uint8_t* vp = a.val + row * a.vstride + (uint64_t)c * a.w;
  for (uint32_t b = 0; b < a.w; b++) vp[b] = (uint8_t)(be >> (8 * (a.w - 1 - b)));
}

}  // namespace tsdb

namespace tsdb {
// An empty integer min / max partial (count 0) as the neutral element of the
// rank allreduce (acc_merge skips empty partials; a reduction cannot).
__global__ void k_neutral_minmax(const uint32_t* cnt, int64_t* v, uint64_t T, int64_t neutral) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g < T && cnt[g] == 0) v[g] = neutral;
}

__global__ void k_bitmap_or(const uint32_t* all, uint32_t nranks, uint64_t nwords, uint32_t* out) {
  const uint64_t w = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (w >= nwords) return;
  uint32_t x = 0;
  for (uint32_t r = 0; r < nranks; r++) x |= all[(uint64_t)r * nwords + w];
  out[w] = x;
}
}  // namespace tsdb

namespace tsdb {
// ---- bandwidth probes (achievable bandwidth beside peak) ----
// Streaming read with k_ds_spans' geometry: one wave per span, the span's
// qualifier and value rows read with 16-B loads, 8 cells per lane, one
// chunk in flight while the previous one is folded (XOR) into a register.
__global__ void __launch_bounds__(256) k_probe_read(const uint64_t* span_row_start, const uint32_t* ncells,
                                                    const uint64_t* qoff, const uint64_t* voff, const uint8_t* qual,
                                                    const uint8_t* val, uint32_t n_spans, uint32_t w,
                                                    uint32_t* sink) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  uint32_t acc = 0;
  for (uint32_t s = wave; s < n_spans; s += nwaves) {
    for (uint64_t r = span_row_start[s]; r < span_row_start[s + 1]; r++) {
      const uint32_t nc = ncells[r];
      const uint8_t* q = qual + qoff[r];
      const uint8_t* v = val + voff[r];
      for (uint32_t c0 = 0; c0 < nc; c0 += 512) {
        const uint32_t c = c0 + 8u * lane;
        if (c < nc) {
          const uint4 a = *(const uint4*)(q + 2ull * c);
          acc ^= a.x ^ a.y ^ a.z ^ a.w;
          for (uint32_t i = 0; i < 2 * w / 4; i++) {
            const uint4 b = *(const uint4*)(v + (uint64_t)w * c + 16ull * i);
            acc ^= b.x ^ b.y ^ b.z ^ b.w;
          }
        }
      }
    }
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;  // keeps the loads alive
}

// Device copy, 16 B per lane per iteration (grid-stride).
__global__ void __launch_bounds__(256) k_probe_copy(const uint4* src, uint4* dst, uint64_t n16) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// Flat streaming read of [p, p + n16*16): 4 x 16 B per lane in flight per
// iteration, grid-stride (the pure-read ceiling of the box).
__global__ void __launch_bounds__(256) k_probe_flat(const uint4* p, uint64_t n16, uint32_t* sink) {
  uint32_t acc = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n16; i += 4 * stride) {
    const uint4 a = p[i], b = p[i + stride], c = p[i + 2 * stride], d = p[i + 3 * stride];
    acc ^= a.x ^ b.y ^ c.z ^ d.w;
  }
  for (; i < n16; i += stride) acc ^= p[i].x;
  if (acc == 0x9e3779b9u) sink[0] = acc;
}

// k_probe_read with two chunks in flight per wave and the next span's row
// metadata loaded while the current span streams (single-row spans).
__global__ void __launch_bounds__(256) k_probe_read2(const uint64_t* span_row_start, const uint32_t* ncells,
                                                     const uint64_t* qoff, const uint64_t* voff,
                                                     const uint8_t* qual, const uint8_t* val, uint32_t n_spans,
                                                     uint32_t* sink) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  uint32_t acc = 0;
  uint32_t s = wave;
  if (s >= n_spans) return;
  uint64_t r = span_row_start[s];
  uint32_t nc = ncells[r];
  uint64_t qo = qoff[r], vo = voff[r];
  for (; s < n_spans; s += nwaves) {
    const uint32_t sn = s + nwaves;
    uint64_t rn = 0, qn = 0, vn = 0;
    uint32_t ncn = 0;
    if (sn < n_spans) {
      rn = span_row_start[sn];
      ncn = ncells[rn];
      qn = qoff[rn];
      vn = voff[rn];
    }
    const uint8_t* q = qual + qo;
    const uint8_t* v = val + vo;
    for (uint32_t c0 = 0; c0 < nc; c0 += 1024) {
      const uint32_t c = c0 + 8u * lane, c2 = c + 512;
      uint4 a = {0, 0, 0, 0}, b[4] = {}, a2 = {0, 0, 0, 0}, b2[4] = {};
      if (c < nc) {
        a = *(const uint4*)(q + 2ull * c);
        for (int i = 0; i < 4; i++) b[i] = *(const uint4*)(v + 8ull * c + 16ull * i);
      }
      if (c2 < nc) {
        a2 = *(const uint4*)(q + 2ull * c2);
        for (int i = 0; i < 4; i++) b2[i] = *(const uint4*)(v + 8ull * c2 + 16ull * i);
      }
      acc ^= a.x ^ a.y ^ a.z ^ a.w ^ a2.x ^ a2.w;
      for (int i = 0; i < 4; i++) acc ^= b[i].x ^ b[i].w ^ b2[i].y ^ b2[i].z;
    }
    nc = ncn;
    qo = qn;
    vo = vn;
  }
  if (acc == 0x9e3779b9u) sink[0] = acc;
}
}  // namespace tsdb
