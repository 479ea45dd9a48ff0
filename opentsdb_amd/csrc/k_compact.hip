// k_compact.hip — CompactionQueue.compact(row, compacted) on gfx950
// (reference: src/core/CompactionQueue.java:243-743), the secondary path.
//
// Two launches over a batch of rows (tsdbhip_rows_desc):
//   k_compact_rows     one wave per row (grid-stride). Reads the KV lengths
//                      and the 2-byte qualifiers, classifies the row exactly
//                      as compact() does (junk KVs, single KV, the in-order
//                      delta check of the trivial pre-pass :286-333, legacy
//                      floats) and writes single / trivial / error rows
//                      directly. Rows holding a compacted cell (complex) go
//                      to a work list.
//   k_compact_complex  one 256-thread block per complex row: breakDownValues
//                      (:690-743) into a cell table (LDS, or global scratch
//                      for rows over LDS_CELLS cells), then the stable sort +
//                      duplicate check of complexCompact (:600-679) as a
//                      4096-slot table indexed by the 12-bit time delta:
//                      slot[delta] = first cell (atomicMin); every other cell
//                      of that delta must equal it byte for byte (same
//                      q[1], same value) or the row is an
//                      IllegalDataException. Emission walks the slots in
//                      delta order, which is the sorted order.
// Output placement needs no scan: row r writes at its input qualifier offset
// and at its input value offset + r (include/tsdbhip.h). Byte work, HBM-bound;
// no MFMA.
#pragma once
#include "dev_common.h"

namespace tsdb {

constexpr uint32_t CQ_LDS_CELLS = 6144;  // cells per complex row held in LDS
constexpr uint32_t CQ_SLOTS = 4096;      // 12-bit time deltas (Const.java:26)

// row status (include/tsdbhip.h)
constexpr uint8_t CQ_NONE = 0, CQ_SINGLE = 1, CQ_TRIVIAL = 2, CQ_COMPLEX = 3, CQ_ERROR = 4, CQ_OOB = 5;

struct CompactArgs {
  uint64_t n_rows, n_kvs;
  const uint64_t* row_kv_start;
  const uint64_t* row_qual_off;
  const uint64_t* row_val_off;
  const uint16_t* kv_qual_len;
  const uint16_t* kv_val_len;
  const uint8_t* qual;
  const uint8_t* val;
  uint64_t qual_nbytes, val_nbytes;
  uint64_t qcap, vcap;
  uint8_t* status;
  uint64_t* out_qoff;
  uint32_t* out_qlen;
  uint64_t* out_voff;
  uint32_t* out_vlen;
  uint8_t* oq;
  uint8_t* ov;
  uint32_t* counters;   // [0] complex rows in LDS list, [1] in big list, [2] bad-argument flag
  uint32_t* list_lds;   // complex rows with <= CQ_LDS_CELLS cells
  uint32_t* list_big;   // the others
  uint64_t* big_cells;  // scratch: row r's cells at (row_qual_off[r]-row_qual_off[0])/2 + r
};

// fixQualifierFlags (CompactionQueue.java:490-499), byte arithmetic.
DEVI uint32_t cq_fixq(uint32_t flags, uint32_t vlen) { return ((flags & ~7u) | (vlen - 1u)) & 0xFFu; }
// floatingPointValueToFix (:510-515).
DEVI bool cq_legacy(uint32_t flags, uint32_t vlen) { return (flags & 8u) && (flags & 7u) == 3u && vlen == 8u; }
DEVI uint32_t ld_q16(const uint8_t* p, uint64_t off) { return ((uint32_t)p[off] << 8) | p[off + 1]; }

struct RowHdr {
  uint64_t kb, nk, qs, qe, vs, ve, oqo, ovo;
  bool ok;
};

DEVI RowHdr cq_row(const CompactArgs& a, uint64_t r) {
  RowHdr h;
  h.kb = a.row_kv_start[r];
  const uint64_t ke = a.row_kv_start[r + 1];
  h.qs = a.row_qual_off[r];
  h.qe = a.row_qual_off[r + 1];
  h.vs = a.row_val_off[r];
  h.ve = a.row_val_off[r + 1];
  const uint64_t q0 = a.row_qual_off[0], v0 = a.row_val_off[0];
  h.ok = h.kb <= ke && ke <= a.n_kvs && h.qs <= h.qe && h.qe <= a.qual_nbytes && h.vs <= h.ve &&
         h.ve <= a.val_nbytes && h.qs >= q0 && h.vs >= v0 && (h.ve - h.vs) < (1ull << 32);
  h.nk = h.ok ? ke - h.kb : 0;
  h.oqo = h.qs - q0;
  h.ovo = h.vs - v0 + r;
  h.ok = h.ok && h.oqo + (h.qe - h.qs) <= a.qcap && h.ovo + (h.ve - h.vs) + 1 <= a.vcap;
  return h;
}

DEVI void cq_finish(const CompactArgs& a, uint64_t r, uint8_t st, uint32_t qlen, uint32_t vlen) {
  a.status[r] = st;
  a.out_qlen[r] = qlen;
  a.out_vlen[r] = vlen;
}

// Wave copy of n bytes, lanes striding (coalesced on both sides).
DEVI void wave_copy(uint8_t* dst, const uint8_t* src, uint64_t n, int lane) {
  for (uint64_t j = lane; j < n; j += WAVE) dst[j] = src[j];
}

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256) k_compact_rows(CompactArgs a) {
  const int lane = lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * blockDim.x / WAVE;
  for (uint64_t r = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) / WAVE; r < a.n_rows; r += nwaves) {
    const RowHdr h = cq_row(a, r);
    if (lane == 0) {
      a.out_qoff[r] = h.oqo;
      a.out_voff[r] = h.ovo;
    }
    // ---- pass 1: classify (CompactionQueue.java:244-333) ----
    uint64_t qcar = 0, vcar = 0, ncells = 0;
    uint32_t nvalid = 0, nmulti = 0;
    int last_delta = -1;
    bool err_delta = false, legacy_bad = false, any_legacy = false, any_junk = false;
    uint64_t f_qpos = 0, f_vpos = 0;
    uint32_t f_ql = 0, f_vl = 0, f_q = 0;
    for (uint64_t base = 0; base < h.nk; base += WAVE) {
      const uint64_t i = base + lane;
      const bool act = i < h.nk;
      const uint32_t ql = act ? a.kv_qual_len[h.kb + i] : 0u;
      const uint32_t vl = act ? a.kv_val_len[h.kb + i] : 0u;
      const uint32_t qi = wave_incl_scan_u32_dpp(ql), vi = wave_incl_scan_u32_dpp(vl);
      const uint64_t qpos = h.qs + qcar + (qi - ql), vpos = h.vs + vcar + (vi - vl);
      qcar += readlane_u32(qi, 63);
      vcar += readlane_u32(vi, 63);
      const bool valid = act && ql != 0 && (ql & 1) == 0;
      const bool two = valid && ql == 2;
      const bool inq = qpos + ql <= h.qe, inv = vpos + vl <= h.ve;
      const uint32_t q = (two && inq) ? ld_q16(a.qual, qpos) : 0u;
      const int delta = (int)(q >> 4);
      const bool leg = two && cq_legacy(q & 0xFF, vl);
      bool lbad = false;
      if (leg && inv) lbad = (a.val[vpos] | a.val[vpos + 1] | a.val[vpos + 2] | a.val[vpos + 3]) != 0;
      // delta strictly increasing over the 2-byte KVs, in input order (:317-328)
      const uint64_t m2 = ballot(two);
      const uint64_t lower = m2 & lanemask_lt(lane);
      const int pl = lower ? 63 - __clzll(lower) : lane;
      int pd = __shfl(delta, pl);
      if (!lower) pd = last_delta;
      err_delta |= ballot(two && delta <= pd) != 0;
      if (m2) last_delta = __shfl(delta, 63 - __clzll(m2));
      legacy_bad |= ballot(lbad) != 0;
      any_legacy |= ballot(leg) != 0;
      any_junk |= ballot(act && !valid) != 0;
      const uint64_t mv = ballot(valid);
      if (nvalid == 0 && mv) {
        const int fl = __ffsll((long long)mv) - 1;
        f_qpos = readlane_u64(qpos, fl);
        f_vpos = readlane_u64(vpos, fl);
        f_ql = readlane_u32(ql, fl);
        f_vl = readlane_u32(vl, fl);
        f_q = readlane_u32(q, fl);
      }
      nvalid += __popcll(mv);
      nmulti += __popcll(ballot(valid && ql > 2));
      ncells += readlane_u32(wave_incl_scan_u32_dpp(valid ? ql >> 1 : 0u), 63);
    }
    if (!h.ok || qcar != h.qe - h.qs || vcar != h.ve - h.vs) {
      if (lane == 0) {
        atomicOr(&a.counters[2], 1u);
        cq_finish(a, r, CQ_NONE, 0, 0);
      }
      continue;
    }
    if (nvalid == 0) {  // empty row, or only junk (:245-247, :301-306, :335-337)
      if (lane == 0) cq_finish(a, r, CQ_NONE, 0, 0);
      continue;
    }
    if (nvalid == 1) {  // one KV (left): compacted[0] = kv, float-fixed (:248-266)
      if (f_ql == 2 && cq_legacy(f_q & 0xFF, f_vl)) {
        const bool bad = (a.val[f_vpos] | a.val[f_vpos + 1] | a.val[f_vpos + 2] | a.val[f_vpos + 3]) != 0;
        if (bad) {
          if (lane == 0) cq_finish(a, r, CQ_ERROR, 0, 0);
        } else {
          if (lane < 4) a.ov[h.ovo + lane] = a.val[f_vpos + 4 + lane];
          if (lane == 0) {
            a.oq[h.oqo] = (uint8_t)(f_q >> 8);
            a.oq[h.oqo + 1] = (uint8_t)cq_fixq(f_q & 0xFF, 4);
            cq_finish(a, r, CQ_SINGLE, 2, 4);
          }
        }
      } else {
        wave_copy(a.oq + h.oqo, a.qual + f_qpos, f_ql, lane);
        wave_copy(a.ov + h.ovo, a.val + f_vpos, f_vl, lane);
        if (lane == 0) cq_finish(a, r, CQ_SINGLE, f_ql, f_vl);
      }
      continue;
    }
    if (err_delta || (nmulti == 0 && legacy_bad)) {  // :324-327, fixFloatingPointValue :538
      if (lane == 0) cq_finish(a, r, CQ_ERROR, 0, 0);
      continue;
    }
    if (nmulti) {  // complexCompact: handed to k_compact_complex
      if (lane == 0) {
        if (ncells <= CQ_LDS_CELLS) a.list_lds[atomicAdd(&a.counters[0], 1u)] = (uint32_t)r;
        else a.list_big[atomicAdd(&a.counters[1], 1u)] = (uint32_t)r;
      }
      continue;
    }
    // ---- trivialCompact (:450-474): q[0], fixed q[1]; fixed values; 0x00 ----
    if (!any_legacy && !any_junk) {
      // values pass through unchanged: one coalesced copy of the row's values
      wave_copy(a.ov + h.ovo, a.val + h.vs, h.ve - h.vs, lane);
    }
    uint64_t qc2 = 0, vc2 = 0, nq = 0, nv = 0;
    for (uint64_t base = 0; base < h.nk; base += WAVE) {
      const uint64_t i = base + lane;
      const bool act = i < h.nk;
      const uint32_t ql = act ? a.kv_qual_len[h.kb + i] : 0u;
      const uint32_t vl = act ? a.kv_val_len[h.kb + i] : 0u;
      const uint32_t qi = wave_incl_scan_u32_dpp(ql), vi = wave_incl_scan_u32_dpp(vl);
      const uint64_t qpos = h.qs + qc2 + (qi - ql), vpos = h.vs + vc2 + (vi - vl);
      qc2 += readlane_u32(qi, 63);
      vc2 += readlane_u32(vi, 63);
      const bool valid = act && ql == 2;
      const uint32_t q = valid ? ld_q16(a.qual, qpos) : 0u;
      const bool leg = valid && cq_legacy(q & 0xFF, vl);
      const uint32_t flen = valid ? (leg ? 4u : vl) : 0u;
      const uint64_t mv = ballot(valid);
      const uint32_t rank = __popcll(mv & lanemask_lt(lane));
      const uint32_t fi = wave_incl_scan_u32_dpp(flen);
      if (valid) {
        const uint64_t oq = h.oqo + 2 * (nq + rank);
        a.oq[oq] = (uint8_t)(q >> 8);
        a.oq[oq + 1] = (uint8_t)cq_fixq(q & 0xFF, flen);
        if (any_legacy || any_junk) {
          const uint64_t src = vpos + (leg ? 4 : 0), dst = h.ovo + nv + (fi - flen);
          for (uint32_t j = 0; j < flen; j++) a.ov[dst + j] = a.val[src + j];
        }
      }
      nq += __popcll(mv);
      nv += readlane_u32(fi, 63);
    }
    if (lane == 0) {
      a.ov[h.ovo + nv] = 0;
      cq_finish(a, r, CQ_TRIVIAL, (uint32_t)(2 * nq), (uint32_t)(nv + 1));
    }
  }
}

// ---------------------------------------------------------------------------
// Block (256 threads = 4 waves) exclusive scan of two u32 values.
DEVI void block_excl_scan2(uint32_t x, uint32_t y, uint32_t& ex, uint32_t& ey, uint32_t& tx, uint32_t& ty,
                           uint32_t* sh /* [8] */) {
  const int lane = lane_id(), w = threadIdx.x / WAVE;
  const uint32_t ix = wave_incl_scan_u32_dpp(x), iy = wave_incl_scan_u32_dpp(y);
  __syncthreads();  // sh reuse
  if (lane == 63) {
    sh[w] = ix;
    sh[4 + w] = iy;
  }
  __syncthreads();
  uint32_t px = 0, py = 0;
  tx = ty = 0;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    if (k < w) {
      px += sh[k];
      py += sh[4 + k];
    }
    tx += sh[k];
    ty += sh[4 + k];
  }
  ex = px + ix - x;
  ey = py + iy - y;
}

struct MultiEnt {
  uint64_t qpos, vpos;
  uint32_t kv, vl, nc, cb;
};

// cell word: q (16) | len (16) | value offset relative to the row's values (32)
DEVI uint64_t cq_cell(uint32_t q, uint32_t len, uint32_t off) {
  return ((uint64_t)q << 48) | ((uint64_t)(len & 0xFFFF) << 32) | off;
}

template <bool kLds>
__global__ void __launch_bounds__(256) k_compact_complex(CompactArgs a) {
  __shared__ uint32_t slot[CQ_SLOTS];
  __shared__ uint64_t lcells[kLds ? CQ_LDS_CELLS : 1];
  __shared__ MultiEnt multi[256];
  __shared__ uint32_t sh_scan[8];
  __shared__ uint32_t n_multi, err_kv, dmin, dmax;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
  const uint32_t n = a.counters[kLds ? 0 : 1];
  const uint32_t* list = kLds ? a.list_lds : a.list_big;
  for (uint32_t wi = blockIdx.x; wi < n; wi += gridDim.x) {
    const uint64_t r = list[wi];
    const RowHdr h = cq_row(a, r);
    uint64_t* cells = kLds ? lcells : a.big_cells + h.oqo / 2 + r;
    for (int d = tid; d < (int)CQ_SLOTS; d += 256) slot[d] = ~0u;
    if (tid == 0) {
      n_multi = 0;
      err_kv = ~0u;
      dmin = CQ_SLOTS - 1;
      dmax = 0;
    }
    __syncthreads();
    // ---- breakDownValues (:690-743), KVs in chunks of 256 ----
    uint64_t qcar = 0, vcar = 0, ccar = 0;
    for (uint64_t base = 0; base < h.nk; base += 256) {
      const uint64_t i = base + tid;
      const bool act = i < h.nk;
      const uint32_t ql = act ? a.kv_qual_len[h.kb + i] : 0u;
      const uint32_t vl = act ? a.kv_val_len[h.kb + i] : 0u;
      const bool valid = act && ql != 0 && (ql & 1) == 0;
      const uint32_t nc = valid ? ql >> 1 : 0u;
      uint32_t qx, vx, tq, tv, cx, tc, dummy, td;
      block_excl_scan2(ql, vl, qx, vx, tq, tv, sh_scan);
      block_excl_scan2(nc, 0u, cx, dummy, tc, td, sh_scan);
      const uint64_t qpos = h.qs + qcar + qx, vpos = h.vs + vcar + vx;
      const uint32_t cb = (uint32_t)(ccar + cx);
      if (valid && ql == 2) {
        const uint32_t q = ld_q16(a.qual, qpos);
        const bool leg = cq_legacy(q & 0xFF, vl);
        if (leg && (a.val[vpos] | a.val[vpos + 1] | a.val[vpos + 2] | a.val[vpos + 3]) != 0)
          atomicMin(&err_kv, (uint32_t)(i << 1));  // IllegalDataException (:538)
        const uint32_t flen = leg ? 4u : vl;
        cells[cb] = cq_cell((q & 0xFF00) | cq_fixq(q & 0xFF, flen), flen,
                            (uint32_t)(vpos - h.vs) + (leg ? 4u : 0u));
      } else if (valid) {
        const uint32_t e = atomicAdd(&n_multi, 1u);
        multi[e] = MultiEnt{qpos, vpos, (uint32_t)i, vl, nc, cb};
      }
      __syncthreads();
      const uint32_t nm = n_multi;
      for (uint32_t e = w; e < nm; e += 4) {  // one wave per multi-value cell
        const MultiEnt m = multi[e];
        if (m.vl == 0) {  // val[val.length - 1] on an empty value (:708)
          if (lane == 0) atomicMin(&err_kv, (m.kv << 1) | 1u);
          continue;
        }
        if (a.val[m.vpos + m.vl - 1] != 0) {  // unknown meta byte (:709-714)
          if (lane == 0) atomicMin(&err_kv, m.kv << 1);
          continue;
        }
        uint32_t run = 0;
        bool over = false;
        for (uint32_t c0 = 0; c0 < m.nc; c0 += WAVE) {
          const uint32_t c = c0 + lane;
          const bool a2 = c < m.nc;
          const uint32_t q = a2 ? ld_q16(a.qual, m.qpos + 2ull * c) : 0u;
          const uint32_t len = a2 ? (q & 7u) + 1u : 0u;
          const uint32_t incl = wave_incl_scan_u32_dpp(len);
          const uint32_t off = run + incl - len;
          if (a2) {
            over |= off + len > m.vl;  // System.arraycopy past the value (:722)
            cells[m.cb + c] = cq_cell(q, len, (uint32_t)(m.vpos - h.vs) + off);
          }
          run += readlane_u32(incl, 63);
        }
        if (ballot(over)) {
          if (lane == 0) atomicMin(&err_kv, (m.kv << 1) | 1u);
        } else if (run != m.vl - 1) {  // did not consume the value (:730-736)
          if (lane == 0) atomicMin(&err_kv, m.kv << 1);
        }
      }
      __syncthreads();
      if (tid == 0) n_multi = 0;
      qcar += tq;
      vcar += tv;
      ccar += tc;
    }
    __syncthreads();
    const uint32_t ncells = (uint32_t)ccar;
    if (err_kv != ~0u) {
      if (tid == 0) cq_finish(a, r, (err_kv & 1u) ? CQ_OOB : CQ_ERROR, 0, 0);
      __syncthreads();
      continue;
    }
    // ---- sort + duplicate check (:606-650) via the delta slot table ----
    for (uint32_t c = tid; c < ncells; c += 256) {
      const uint32_t d = (uint32_t)(cells[c] >> 52);
      atomicMin(&slot[d], c);
      atomicMin(&dmin, d);
      atomicMax(&dmax, d);
    }
    __syncthreads();
    bool bad = false;
    for (uint32_t c = tid; c < ncells; c += 256) {
      const uint64_t cw = cells[c];
      const uint32_t rep = slot[cw >> 52];
      if (rep == c) continue;
      const uint64_t rw = cells[rep];
      const uint32_t len = (uint32_t)(cw >> 32) & 0xFFFF;
      if (((cw >> 48) & 0xFF) != ((rw >> 48) & 0xFF) || len != (((uint32_t)(rw >> 32)) & 0xFFFF)) {
        bad = true;
        continue;
      }
      const uint8_t* x = a.val + h.vs + (uint32_t)cw;
      const uint8_t* y = a.val + h.vs + (uint32_t)rw;
      for (uint32_t j = 0; j < len; j++) bad |= x[j] != y[j];
    }
    if (__syncthreads_or(bad)) {
      if (tid == 0) cq_finish(a, r, CQ_ERROR, 0, 0);
      __syncthreads();
      continue;
    }
    // ---- emit in delta order: qualifiers || values || 0x00 (:652-678) ----
    uint64_t nq = 0, nv = 0;
    const uint32_t d_lo = dmin, d_hi = dmax;
    for (uint32_t d0 = d_lo; d0 <= d_hi; d0 += 256) {
      const uint32_t d = d0 + tid;
      const uint32_t rep = d <= d_hi ? slot[d] : ~0u;
      const bool present = rep != ~0u;
      const uint64_t cw = present ? cells[rep] : 0ull;
      const uint32_t len = present ? ((uint32_t)(cw >> 32) & 0xFFFF) : 0u;
      uint32_t rk, vo, tp, tl;
      block_excl_scan2(present ? 1u : 0u, len, rk, vo, tp, tl, sh_scan);
      if (present) {
        const uint64_t oq = h.oqo + 2 * (nq + rk);
        a.oq[oq] = (uint8_t)(cw >> 56);
        a.oq[oq + 1] = (uint8_t)(cw >> 48);
        const uint8_t* src = a.val + h.vs + (uint32_t)cw;
        uint8_t* dst = a.ov + h.ovo + nv + vo;
        for (uint32_t j = 0; j < len; j++) dst[j] = src[j];
      }
      nq += tp;
      nv += tl;
    }
    if (tid == 0) {
      a.ov[h.ovo + nv] = 0;
      cq_finish(a, r, CQ_COMPLEX, (uint32_t)(2 * nq), (uint32_t)(nv + 1));
    }
    __syncthreads();
  }
}

}  // namespace tsdb
