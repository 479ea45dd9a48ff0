// k_direct.hip — the no-downsampling path for spans whose points are a
// regular cadence run of the union grid (the common shape of TSD data:
// every series written at the same fixed interval). For such a span the
// SGIterator never interpolates (SpanGroup.java:702-730: x == x0 at every
// emission time inside [first, last]) and its rate is the span's own
// constant-step difference (SpanGroup.java:741-755), so the reducer can read
// each value straight from the reference's value bytes: no E sequence is
// materialised and the union grid is marked from (x0, step, n) alone.
//
// k_direct_scan (wave per kept span) streams the span's qualifiers only
// (2 B/cell) and proves: uniform value width over all rows (8 or 4 B, the
// reference's write paths, TSDB.java:285,321), one cell type over the
// emitted points, ts strictly on x0 + i*step, no point after `end`, no
// dropped/merged-quirk rows (Q1, the short overflow). It then marks the
// span's grid points. k_direct_verify (thread per candidate, after the grid
// is built) keeps a span direct iff its grid points are consecutive grid
// ranks (no other span puts a point between two of its points, which would
// need a lerp). Spans that fail either test go to the E path (k_decode_*).
#pragma once
#include "dev_common.h"
#include "k_decode.hip"
#include "k_grid.hip"

namespace tsdb {

enum { DIR_ON = 1u, DIR_FLT = 2u, DIR_W8 = 4u, DIR_MULTI = 8u };

struct DirectArgs {
  uint32_t* info;      // [n_kept] DIR_* bits (0: E path)
  uint32_t* n;         // [n_kept] emitted points (cells with ts >= start)
  uint32_t* x0;        // [n_kept] first emitted ts
  uint32_t* step;      // [n_kept] cadence (0 when n == 1)
  uint64_t* voff;      // [n_kept] value byte offset of E[0] (rows of E[0])
  uint32_t* c0;        // [n_kept] span cell index of E[0]
  uint64_t* r0;        // [n_kept] first row of the span
  uint32_t* ga;        // [n_kept] grid rank of the span's first grid point
  uint32_t* row_cpre;  // [R] span-local index of each row's first cell
  uint32_t* list;      // spans left to the E path
  uint32_t* list_count;
  uint32_t* bitmap;
  const uint32_t* word_rank;
  int64_t lo, hi;
  int32_t rate;
  uint32_t batch;      // spans per wave batch (<= DIRB): fewer for small groups, so
                       // they spread over more waves
  // the lockstep proposal of k_direct_opt (null: none made): the spans'
  // class keys [min, max] of (x0 << 32 | n) and of (step << 32 | q0), and the
  // count of kept spans outside any class
  const unsigned long long* ls_key;
  const uint32_t* ls_other;
};

// ---- the lockstep proposal (k_lockstep.hip) ----
// A span of one row with n >= 2 cells of one width W (8 or 4 B) whose
// qualifiers at cells 0, 1 and n-1 agree with ts = x0 + c*step (same flags),
// every point inside [start, end], proposes the class key (x0 << 32 | n,
// step << 32 | q0); k_lockstep proves every other qualifier while it reduces.
DEVI bool ls_probe(const DecodeArgs& a, const uint32_t* ncells, const uint32_t* vlen, uint32_t k, uint64_t& k1,
                   uint64_t& k2, uint64_t& r0_out, uint64_t& qo_out, uint64_t& vo_out) {
  const uint32_t s = a.kept[k];
  const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
  const uint32_t n = a.sp_ncells[s];
  if (!(r1 - r0 == 1 && n >= 2 && a.sp_q1[s] < 0 && a.sp_ovf_cell[s] < 0 && a.row_ok[r0] && ncells[r0] == n))
    return false;
  const uint32_t vb = vlen[r0] - 1;  // (n >= 2: a compacted row ends with its meta byte)
  const uint32_t W = vb / n;
  const uint64_t qo = a.row_qual_off[r0], vo = a.row_val_off[r0];
  if (!((W == 8 || W == 4) && vb == W * n && (qo & 1) == 0 && (vo & (W - 1)) == 0)) return false;
  const uint32_t q0 = load_qual(a.qual, qo), q1 = load_qual(a.qual, qo + 2), ql = load_qual(a.qual, qo + 2ull * (n - 1));
  const uint32_t fl = q0 & 15u;
  const uint32_t d0 = q0 >> 4, d1 = q1 >> 4, dl = ql >> 4;
  if (!((fl & 7u) == W - 1 && (q1 & 15u) == fl && (ql & 15u) == fl && d1 > d0 &&
        (uint64_t)d0 + (uint64_t)(n - 1) * (d1 - d0) == dl))
    return false;
  const uint32_t step = d1 - d0;
  const int64_t first = (int64_t)a.row_base[r0] + d0;
  const int64_t last = first + (int64_t)(n - 1) * step;
  if (!(first >= a.start && last <= a.end && last < (1ll << 32))) return false;
  k1 = ((uint64_t)first << 32) | n;
  k2 = ((uint64_t)step << 32) | q0;
  r0_out = r0;
  qo_out = qo;
  vo_out = vo;
  return true;
}

// Lane per kept span: the proposal, and for a proposing span the direct-path
// record k_direct_scan would write for it. The group is lockstep iff every
// span proposes kept span 0's key: each wave compares its spans with that key
// (span 0's probe, repeated by every wave: the same cached lines) and a wave
// that finds a span off it stores 1 to n_other; block 0 publishes the key as
// [min, max] pairs. No atomic, no read of a shared word (every wave polling
// one word across the XCDs' L2s cost more than the probe itself).
__global__ void __launch_bounds__(256) k_direct_opt(DecodeArgs a, DirectArgs g, const uint32_t* ncells,
                                                    const uint32_t* vlen, uint64_t* qoff_out,
                                                    unsigned long long* key, uint32_t* n_other) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (a.n_kept == 0) return;
  uint64_t k1 = 0, k2 = 0, r0 = 0, qo = 0, vo = 0;
  bool cand = false;
  if (k < a.n_kept) {
    cand = ls_probe(a, ncells, vlen, k, k1, k2, r0, qo, vo);
    if (cand) {
      const uint32_t n = (uint32_t)k1, q0 = (uint32_t)k2 & 0xFFFFu;
      g.info[k] = DIR_ON | ((q0 & 8u) ? DIR_FLT : 0u) | ((q0 & 7u) == 7u ? DIR_W8 : 0u);
      g.n[k] = n;
      g.x0[k] = (uint32_t)(k1 >> 32);
      g.step[k] = (uint32_t)(k2 >> 32);
      g.voff[k] = vo;
      g.c0[k] = 0;
      g.r0[k] = r0;
      g.row_cpre[r0] = 0;
      qoff_out[k] = qo;
      a.e_len[k] = n;
      a.e_bad[k] = -1;
    }
  }
  // kept span 0's key (uniform: every lane probes the same span)
  uint64_t z1 = 0, z2 = 0, zr, zq, zv;
  const bool zc = ls_probe(a, ncells, vlen, 0u, z1, z2, zr, zq, zv);
  const bool off = k < a.n_kept && (!cand || k1 != z1 || k2 != z2);
  const int lane = lane_id();
  if (zc && ballot(off) && lane == 0) *(volatile uint32_t*)n_other = 1u;
  if (k == 0) {  // (block 0, lane 0: span 0's own probe decides when it proposes nothing)
    if (!zc) *(volatile uint32_t*)n_other = 1u;
    else {
      key[0] = key[1] = z1;
      key[2] = key[3] = z2;
    }
  }
}

// The group is lockstep: one class key over every kept span (read after
// k_direct_opt, the same on every wave).
DEVI bool ls_lockstep(const DirectArgs& g) {
  if (!g.ls_key) return false;  // (plain loads: written by the previous kernel)
  const unsigned long long* k = g.ls_key;
  return *g.ls_other == 0 && k[0] != ~0ull && k[0] == k[1] && k[2] == k[3];
}

// Marks {xf + p*step : 0 <= p < np} (all inside [lo, hi]) in the grid bitmap;
// a word already holding the bits skips the atomic.
DEVI void direct_mark(const DirectArgs& g, int64_t xf, uint32_t step, uint32_t np) {
  const int lane = lane_id();
  if (np == 0) return;
  if (step >= 32 || np == 1) {
    for (uint32_t p = lane; p < np; p += WAVE) {
      const uint64_t b = (uint64_t)(xf - g.lo) + (uint64_t)p * step;
      const uint32_t bit = 1u << (b & 31);
      uint32_t* w = &g.bitmap[b >> 5];
      if (!(*w & bit)) atomicOr(w, bit);
    }
    return;
  }
  const uint64_t bf = (uint64_t)(xf - g.lo), bl = bf + (uint64_t)(np - 1) * step;
  for (uint64_t w = (bf >> 5) + lane; w <= (bl >> 5); w += WAVE) {
    const uint64_t wb = w << 5;
    uint32_t o = wb >= bf ? (step - (uint32_t)(wb - bf) % step) % step : (uint32_t)(bf - wb);
    uint32_t m = 0;
    for (; o < 32 && wb + o <= bl; o += step) m |= 1u << o;
    if ((g.bitmap[w] & m) != m) atomicOr(&g.bitmap[w], m);
  }
}

// Pending E-path spans of one wave, flushed 64 at a time (one atomic).
struct Pending {
  uint32_t k;    // this lane's slot
  uint32_t cnt;  // uniform
};
DEVI void pend_flush(Pending& p, uint32_t* list, uint32_t* count) {
  if (p.cnt == 0) return;
  const int lane = lane_id();
  uint32_t base = 0;
  if (lane == 0) base = atomicAdd(count, p.cnt);
  base = __builtin_amdgcn_readfirstlane(base);
  if ((uint32_t)lane < p.cnt) list[base + lane] = p.k;
  p.cnt = 0;
}
DEVI void pend_push(Pending& p, uint32_t k, uint32_t* list, uint32_t* count) {
  if (lane_id() == (int)p.cnt) p.k = k;
  if (++p.cnt == WAVE) pend_flush(p, list, count);
}

// A row's qualifier bytes as a buffer resource (range rounded to the 8-byte
// loads; the packer aligns rows to 8 B and buffers carry slack).
DEVI __amdgpu_buffer_rsrc_t qual_rsrc(const uint8_t* p, uint32_t nc) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, 0, (int)((2u * nc + 7u) & ~7u), 0x00020000);
}
DEVI uint2 qload(__amdgpu_buffer_rsrc_t rs, uint32_t voff, uint32_t soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (int)voff, (int)soff, 0);
  return make_uint2(v[0], v[1]);
}

#define DIRB 32           // spans per wave batch (at most)
#define DIRG 8            // groups of 256 cells per wave iteration (4 cells per lane each)
#define DIRQ (256 * DIRG)

// Wave per batch of 64 kept spans: lane l loads span kb+l's metadata and its
// first row's (one dependent-load chain per batch instead of per span), then
// the wave streams the spans one after the other.
__global__ void __launch_bounds__(256) k_direct_scan(DecodeArgs a, DirectArgs g, const uint32_t* ncells,
                                                     const uint32_t* vlen) {
  const int lane = lane_id();
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  if (ls_lockstep(g)) {
    // every span proposed the one key: wave 0 marks its pattern and the
    // group's type (F*: a float series' first point, SpanGroup.java:632-645);
    // the spans' records are k_direct_opt's, their proof is k_lockstep's
    if (wave == 0) {
      const uint64_t k1 = g.ls_key[0], k2 = g.ls_key[2];
      const uint32_t x0 = (uint32_t)(k1 >> 32), n = (uint32_t)k1, step = (uint32_t)(k2 >> 32);
      const bool flt = (k2 & 8u) != 0;
      direct_mark(g, g.rate ? (int64_t)x0 + step : (int64_t)x0, step, g.rate ? n - 1 : n);
      if (lane == 0) {
        atomicOr(&a.gflags[flt ? 0 : 1], 1u);
        if (flt && !a.rate) atomicMax(a.fstar, (unsigned long long)x0 + 1);
      }
    }
    return;
  }
  Pending pend = {0u, 0u};
  bool any_f = false, any_i = false;
  int64_t fs = 0;
  // the last marked pattern (regular series repeat it span after span)
  int64_t m_xf = -1;
  uint32_t m_step = 0, m_np = 0;
  const uint32_t B = g.batch;
  for (uint32_t kb = ufl(wave) * B; kb < a.n_kept; kb += nwaves * B) {
    const uint32_t kl = kb + lane;
    uint32_t s_l = 0, n_l = 0, nc_l = 0, vl_l = 0, base_l = 0;
    uint64_t r0_l = 0, r1_l = 0, qoff_l = 0, voff_l = 0;
    bool ok_l = false;
    if ((uint32_t)lane < B && kl < a.n_kept) {
      s_l = a.kept[kl];
      r0_l = a.span_row_start[s_l];
      r1_l = a.span_row_start[s_l + 1];
      n_l = a.sp_ncells[s_l];
      ok_l = a.sp_q1[s_l] < 0 && a.sp_ovf_cell[s_l] < 0 && n_l > 0 && r1_l > r0_l;
      if (ok_l) {
        nc_l = ncells[r0_l];
        vl_l = vlen[r0_l];
        qoff_l = a.row_qual_off[r0_l];
        voff_l = a.row_val_off[r0_l];
        base_l = a.row_base[r0_l];
        ok_l = a.row_ok[r0_l] != 0 && nc_l > 0;
      }
    }
    const uint32_t nb = min(B, a.n_kept - kb);
    const uint64_t okm = ballot(ok_l);
    // qualifier chunks; the next span's first chunk is loaded while the
    // current span's last chunk is processed (`carry`)
    uint2 cur[DIRG], nxt[DIRG];
    bool carry = false;
    for (uint32_t i = 0; i < nb; i++) {
      const uint32_t k = kb + i;
      const uint64_t r0 = readlane_u64(r0_l, (int)i), r1 = readlane_u64(r1_l, (int)i);
      const uint32_t n = readlane_u32(n_l, (int)i);
      bool ok = (okm >> i) & 1;
      for (uint64_t rb = r0 + 1; ok && rb < r1; rb += WAVE) {  // (uniform loop: `ok` stays scalar)
        const uint64_t r = rb + lane;
        ok = ballot(r < r1 && (a.row_ok[r] == 0 || ncells[r] == 0)) == 0;
      }
      uint32_t W = 0;
      if (ok) {
        const uint32_t nc = readlane_u32(nc_l, (int)i), vl = readlane_u32(vl_l, (int)i);
        const uint32_t vb = nc > 1 ? vl - 1 : vl;
        W = vb == (vb / nc) * nc ? vb / nc : 0;
        ok = W == 8 || W == 4;
      }
      if (!ok) carry = false;
      if (r1 - r0 > WAVE) ok = false;  // (E[0]'s row is found among <= 64 rows)
      // The span is regular iff cell c has ts == first + c*step (u32; the
      // 64-bit `last` check below excludes wrap-around). Per lane: xor of
      // every cell's delta with its expected one, OR / AND of the qualifiers
      // (type and width bits); all reduced once at the span end.
      uint32_t step = 0;       // cadence (0 until two cells were seen)
      uint32_t first = 0;      // ts of cell 0
      uint32_t cell = 0;       // span cell index of the row start
      uint32_t accx = 0, qor = 0, qand = 0xFFFFu;
      uint32_t my_cpre = 0;    // lane j: first span cell of row r0 + j
      bool bad_u = false;      // (uniform)
      for (uint64_t r = r0; ok && r < r1; r++) {
        uint32_t nc, vl, base;
        uint64_t qoff, voff;
        if (r == r0) {
          nc = readlane_u32(nc_l, (int)i);
          vl = readlane_u32(vl_l, (int)i);
          qoff = readlane_u64(qoff_l, (int)i);
          voff = readlane_u64(voff_l, (int)i);
          base = readlane_u32(base_l, (int)i);
        } else {
          nc = ufl(ncells[r]);
          vl = ufl(vlen[r]);
          qoff = ufl64(a.row_qual_off[r]);
          voff = ufl64(a.row_val_off[r]);
          base = ufl(a.row_base[r]);
        }
        const uint32_t vb = nc > 1 ? vl - 1 : vl;
        if (!(vb == W * nc && (qoff & 7) == 0 && (voff & (W - 1)) == 0)) {
          ok = false;
          carry = false;
          break;
        }
        if (lane == 0) g.row_cpre[r] = cell;
        if (lane == (int)(r - r0)) my_cpre = cell;
        // the row's qualifiers through a buffer descriptor: 32-bit offsets with
        // immediate group offsets, and loads past the row return 0 (no clamp)
        const __amdgpu_buffer_rsrc_t rs = qual_rsrc(a.qual + qoff, nc);
        if (!(r == r0 && carry)) {
#pragma unroll
          for (int j = 0; j < DIRG; j++) cur[j] = qload(rs, 8u * lane + 512u * j, 0u);
        }
        carry = false;
        // cadence from the first two cells (lane 0 holds cells 0..3 of the row)
        if (r == r0 || step == 0) {
          const uint32_t w0 = ufl(cur[0].x);
          const uint32_t d0 = (((w0 & 0xFF) << 8) | ((w0 >> 8) & 0xFF)) >> 4;
          const uint32_t d1 = ((((w0 >> 16) & 0xFF) << 8) | (w0 >> 24)) >> 4;
          if (r == r0) {
            first = base + d0;
            if (nc >= 2) step = d1 - d0;
          } else {
            step = base + d0 - first;  // (the first row held one cell)
          }
        }
        const uint32_t lane_off = 4u * (uint32_t)lane * step;
        bool carry_next = false;
        for (uint32_t c0 = 0; c0 < nc; c0 += DIRQ) {
          const uint32_t nc0 = c0 + DIRQ;
          if (nc0 < nc) {
#pragma unroll
            for (int j = 0; j < DIRG; j++) nxt[j] = qload(rs, 8u * lane + 512u * j, 2u * nc0);
          } else if (r + 1 == r1 && i + 1 < nb && ((okm >> (i + 1)) & 1)) {
            const uint64_t nq = readlane_u64(qoff_l, (int)(i + 1));
            const uint32_t nn = readlane_u32(nc_l, (int)(i + 1));
            if ((nq & 7) == 0) {
              const __amdgpu_buffer_rsrc_t ns = qual_rsrc(a.qual + nq, nn);
#pragma unroll
              for (int j = 0; j < DIRG; j++) nxt[j] = qload(ns, 8u * lane + 512u * j, 0u);
              carry_next = true;
            }
          }
#pragma unroll
          for (int j = 0; j < DIRG; j++) {
            const uint32_t g0 = c0 + 256 * j;
            if (g0 >= nc) break;  // (uniform)
            // expected delta of this lane's first cell in the group
            const uint32_t e0 = ufl(first - base + (cell + g0) * step) + lane_off;
            uint32_t q[4];
            q[0] = __builtin_amdgcn_perm(0u, cur[j].x, 0x0C0C0001u);
            q[1] = __builtin_amdgcn_perm(0u, cur[j].x, 0x0C0C0203u);
            q[2] = __builtin_amdgcn_perm(0u, cur[j].y, 0x0C0C0001u);
            q[3] = __builtin_amdgcn_perm(0u, cur[j].y, 0x0C0C0203u);
            // lane's first cell against its expected delta, the next three
            // against their predecessor + step
            if (g0 + 256 <= nc) {  // full group (uniform): no masking
              accx |= (q[0] >> 4) ^ e0;
#pragma unroll
              for (int c = 1; c < 4; c++) accx |= ((q[c] >> 4) - (q[c - 1] >> 4)) ^ step;
#pragma unroll
              for (int c = 0; c < 4; c++) {
                qor |= q[c];
                qand &= q[c];
              }
            } else {
              const uint32_t cl = g0 + 4 * (uint32_t)lane;
              accx |= cl < nc ? (q[0] >> 4) ^ e0 : 0u;
#pragma unroll
              for (int c = 1; c < 4; c++) accx |= cl + c < nc ? ((q[c] >> 4) - (q[c - 1] >> 4)) ^ step : 0u;
#pragma unroll
              for (int c = 0; c < 4; c++) {
                qor |= cl + c < nc ? q[c] : 0u;
                qand &= cl + c < nc ? q[c] : 0xFFFFu;
              }
            }
          }
#pragma unroll
          for (int j = 0; j < DIRG; j++) cur[j] = nxt[j];
        }
        carry = carry_next;
        cell += nc;
      }
      if (n > 1 && step == 0) bad_u = true;  // duplicate timestamps
      // reduce: regular cadence, one width (W), one type
      bool sf = false, si = false;
      if (ok) {
        const bool irregular = ballot(accx != 0) != 0;
        uint32_t wor = 0, wand = 0;  // OR / AND of the qualifiers' low nibble over the span
#pragma unroll
        for (int b = 0; b < 4; b++) {
          if (ballot((qor >> b) & 1)) wor |= 1u << b;
          if (!ballot(!((qand >> b) & 1))) wand |= 1u << b;
        }
        const bool wbad = (wor & 7) != W - 1 || (wand & 7) != W - 1;
        sf = (wor & 8) != 0;
        si = (wand & 8) == 0;
        ok = !irregular && !wbad && !bad_u;
      }
      if (!ok) carry = false;
      uint64_t rz = r0;        // row of E[0]
      uint32_t cpz = 0;        // its first span cell index
      // the emitted points: cells with ts >= start (a suffix), none after end
      uint32_t ne = 0, cz = 0;
      int64_t x0 = 0, last = 0;
      if (ok && cell != n) ok = false;
      if (ok) {
        last = (int64_t)first + (int64_t)(n - 1) * step;
        ok = last <= a.end && last < (1ll << 32);
        if (ok) {
          if ((int64_t)first >= a.start) cz = 0;
          else cz = (uint32_t)min((int64_t)n, ((a.start - (int64_t)first) + step - 1) / (int64_t)max(step, 1u));
          ne = n - cz;
          x0 = (int64_t)first + (int64_t)cz * step;
          ok = ne > 0;
        }
        if (ok) {
          const uint64_t rm = ballot((uint64_t)lane < r1 - r0 && my_cpre <= cz);
          const int hb = 63 - __builtin_clzll(rm);
          rz = r0 + (uint64_t)hb;
          cpz = readlane_u32(my_cpre, hb);
        }
      }
      // one cell type over the emitted points (cells before start do not count:
      // recheck with the type of E cells only when the span mixes)
      if (ok && sf && si) ok = false;
      if (ok) {
        const bool multi = (r1 - rz) > 1;
        const uint32_t info = DIR_ON | (sf ? DIR_FLT : 0u) | (W == 8 ? DIR_W8 : 0u) | (multi ? DIR_MULTI : 0u);
        if (lane == 0) {
          g.info[k] = info;
          g.n[k] = ne;
          g.x0[k] = (uint32_t)x0;
          g.step[k] = ne > 1 ? step : 0u;
          g.voff[k] = a.row_val_off[rz] + (uint64_t)W * (cz - cpz);
          g.c0[k] = cz;
          g.r0[k] = r0;
          a.e_len[k] = ne;
          a.e_bad[k] = -1;
        }
        any_f |= sf;
        any_i |= si;
        if (sf && !a.rate) fs = max(fs, x0 + 1);
        // G: the span's points (rate: from the second)
        const int64_t xf = g.rate ? x0 + step : x0;
        const uint32_t np = g.rate ? ne - 1 : ne;
        if (g.bitmap && np > 0 && !(xf == m_xf && step == m_step && np == m_np)) {
          direct_mark(g, xf, step, np);
          m_xf = xf;
          m_step = step;
          m_np = np;
        }
      } else {
        if (lane == 0) g.info[k] = 0;
        pend_push(pend, k, g.list, g.list_count);
      }
    }
  }
  pend_flush(pend, g.list, g.list_count);
  if (lane == 0) {
    if (any_f && !a.gflags[0]) atomicOr(&a.gflags[0], 1u);
    if (any_i && !a.gflags[1]) atomicOr(&a.gflags[1], 1u);
    if (fs && (unsigned long long)fs > *(volatile unsigned long long*)a.fstar)
      atomicMax(a.fstar, (unsigned long long)fs);
  }
}

// After the grid: keep a candidate direct iff its grid points hold
// consecutive ranks; record the rank of the first. `bsum`: block offsets to
// add to g.word_rank (block-local ranks, k_emit_verify), or null (final ranks).
DEVI void direct_verify_one(const DirectArgs& g, uint32_t n_kept, uint32_t k, const uint32_t* bsum) {
  bool fail = false;
  if (k < n_kept) {
    const uint32_t info = g.info[k];
    if (info & DIR_ON) {
      const uint32_t ne = g.n[k], step = g.step[k];
      const int64_t x0 = g.x0[k];
      const int64_t xf = g.rate ? x0 + step : x0;
      const uint32_t np = g.rate ? ne - 1 : ne;
      if (np == 0) {
        g.ga[k] = 0;  // (rate with one point: inactive everywhere)
      } else {
        const int64_t xl = x0 + (int64_t)(ne - 1) * step;
        const uint32_t ra = bsum ? grid_rank2(g.bitmap, g.word_rank, bsum, g.lo, xf)
                                 : grid_rank(g.bitmap, g.word_rank, g.lo, xf);
        const uint32_t rl = bsum ? grid_rank2(g.bitmap, g.word_rank, bsum, g.lo, xl)
                                 : grid_rank(g.bitmap, g.word_rank, g.lo, xl);
        g.ga[k] = ra;
        if (rl - ra != np - 1) {
          fail = true;
          g.info[k] = 0;
        }
      }
    }
  }
  // wave-aggregated append
  const uint64_t m = ballot(fail);
  if (m) {
    const int lane = lane_id();
    uint32_t base = 0;
    if (lane == __builtin_ctzll(m)) base = atomicAdd(g.list_count, (uint32_t)__popcll(m));
    base = __shfl(base, __builtin_ctzll(m));
    if (fail) g.list[base + __popcll(m & lanemask_lt(lane))] = k;
  }
}

__global__ void __launch_bounds__(256) k_direct_verify(DirectArgs g, uint32_t n_kept) {
  direct_verify_one(g, n_kept, blockIdx.x * blockDim.x + threadIdx.x, nullptr);
}

// k_grid_emit and k_direct_verify in one launch: blocks [0, emit_blocks) emit
// G and write the final word ranks to rank_out; the rest verify the direct
// candidates from the block-local ranks + block offsets (read-only here).
__global__ void __launch_bounds__(256) k_emit_verify(GridArgs ga, uint32_t* rank_out, DirectArgs dg, uint32_t n_kept,
                                                     uint32_t emit_blocks) {
  if (blockIdx.x < emit_blocks) {
    grid_emit_to(ga, (uint64_t)blockIdx.x * 256 + threadIdx.x, rank_out);
  } else {
    direct_verify_one(dg, n_kept, (blockIdx.x - emit_blocks) * 256 + threadIdx.x, ga.block_sum);
  }
}

// Per reduce chunk of spc spans: 1 iff it holds an E span (a span whose
// direct bit is off). A wave per chunk writes every flag (no memset first).
__global__ void __launch_bounds__(256) k_chunk_flags_w(const uint32_t* d_info, uint32_t n_kept, uint32_t spc,
                                                       uint32_t n_chunks, uint32_t* chunk_e) {
  const uint32_t c = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  if (c >= n_chunks) return;
  const uint32_t a = c * spc, b = min(n_kept, a + spc);
  bool any = false;
  for (uint32_t k0 = a; k0 < b && !any; k0 += WAVE) {
    const uint32_t k = k0 + lane_id();
    any = ballot(k < b && !(d_info[k] & 1u)) != 0;
  }
  if (lane_id() == 0) chunk_e[c] = any ? 1u : 0u;
}

}  // namespace tsdb
