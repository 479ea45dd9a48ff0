// k_compact.hip — CompactionQueue.compact(row, compacted) on gfx950
// (reference: src/core/CompactionQueue.java:243-743), the secondary path.
//
// Launches over a batch of rows (tsdbhip_rows_desc):
//   k_compact_tiles    the main kernel (see its comment below): tiles of 16
//                      consecutive rows staged in LDS with 16-B loads; each
//                      wave classifies a row exactly as compact() does (junk
//                      KVs, single KV, the in-order delta check of the trivial
//                      pre-pass :286-333, legacy floats) and compacts it
//                      LDS -> LDS, complex rows of <= 256 cells included;
//                      the tile is written back with 16-B stores.
//                      cq_row_global is the same per-row logic straight from
//                      global memory, for tiles over the LDS budget.
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
constexpr uint8_t CQ_PENDING = 0xFF;  // (k_compact_classify: not plain, for k_compact_rows)

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
  uint8_t* out_write;   // optional (null): tsdb.put decision per row
  int32_t* out_keep;    // optional: KV of the row not to delete, -1 none
  uint32_t* counters;   // [0] complex rows in LDS list, [1] in big list, [2] bad-argument flag,
                        // [3] complex rows finished in-wave by k_compact_tiles
  uint32_t* list_lds;   // complex rows with <= CQ_LDS_CELLS cells
  uint32_t* list_big;   // the others
  uint64_t* big_cells;  // scratch: row r's cells at (row_qual_off[r]-row_qual_off[0])/2 + r
  uint8_t* tile_bad;    // [tile] k_compact_quals skipped the tile (offsets out of bounds)
  uint2* row_holes;     // [row] k_compact_classify: output positions of the first two legacy floats, ~0u none
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

// Row results. Write-back decision: every TRIVIAL row is put (:276; its
// compacted qualifier is longer than any of its KVs'), COMPLEX rows are put
// unless k_compact_dups finds the compacted cell already in the row.
DEVI void cq_finish(const CompactArgs& a, uint64_t r, uint8_t st, uint32_t qlen, uint32_t vlen) {
  a.status[r] = st;
  a.out_qlen[r] = qlen;
  a.out_vlen[r] = vlen;
  if (a.out_write) {
    a.out_write[r] = (st == CQ_TRIVIAL || st == CQ_COMPLEX) ? 1 : 0;
    a.out_keep[r] = -1;
  }
}

// Wave copy of n bytes, lanes striding (coalesced on both sides).
DEVI void wave_copy(uint8_t* dst, const uint8_t* src, uint64_t n, int lane) {
  for (uint64_t j = lane; j < n; j += WAVE) dst[j] = src[j];
}

// ---------------------------------------------------------------------------
// One row by one wave straight from global memory: the fallback of
// k_compact_tiles for tiles that do not fit its LDS budget.
DEVI void cq_row_global(const CompactArgs& a, uint64_t r, int lane) {
  {
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
      return;
    }
    if (nvalid == 0) {  // empty row, or only junk (:245-247, :301-306, :335-337)
      if (lane == 0) cq_finish(a, r, CQ_NONE, 0, 0);
      return;
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
      return;
    }
    if (err_delta || (nmulti == 0 && legacy_bad)) {  // :324-327, fixFloatingPointValue :538
      if (lane == 0) cq_finish(a, r, CQ_ERROR, 0, 0);
      return;
    }
    if (nmulti) {  // complexCompact: handed to k_compact_complex
      if (lane == 0) {
        if (ncells <= CQ_LDS_CELLS) a.list_lds[atomicAdd(&a.counters[0], 1u)] = (uint32_t)r;
        else a.list_big[atomicAdd(&a.counters[1], 1u)] = (uint32_t)r;
      }
      return;
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


// ===========================================================================
// k_compact_tiles: the main compaction kernel. A 256-thread block takes a tile
// of CT_ROWS consecutive rows; their KV lengths, qualifier bytes and value
// bytes are contiguous in the batch, so the block stages them into LDS with
// 16-B loads (one round trip for the whole tile), each wave compacts rows of
// the tile LDS -> LDS, and the block writes the tile's output ranges back with
// 16-B stores (byte stores only at the tile's two edges). Rows holding a
// compacted cell are finished in-wave when they break down into at most
// CT_SORT cells (bitonic sort of (qualifier, cell index) keys = the stable
// Collections.sort of complexCompact, :607); longer ones go to the
// k_compact_complex lists. Tiles over the LDS budget fall back to
// cq_row_global.
// ===========================================================================
constexpr int CT_ROWS = 16;    // rows per tile
constexpr int CT_QB = 4096;    // qualifier bytes per tile
constexpr int CT_VB = 7168;    // value bytes per tile (with CT_KB: k_compact_rows fits 4 blocks per CU)
constexpr int CT_KB = 1280;    // KVs per tile
constexpr int CT_SORT = 256;   // cells of an in-wave complexCompact
constexpr int CQ_RUNS_SLOTS = 12;

struct __attribute__((aligned(16))) TileLds {
  uint8_t qin[CT_QB + 32];
  uint8_t vin[CT_VB + 32];
  uint8_t qout[CT_QB + 32];
  uint8_t vout[CT_VB + 32 + CT_ROWS];
  uint8_t qlen[2 * CT_KB + 32];
  uint8_t vlen[2 * CT_KB + 32];
  uint32_t keys[4][CT_SORT];
  uint32_t pay[4][CT_SORT];
  uint32_t runs[4][CQ_RUNS_SLOTS];
  uint64_t hdr[3][CT_ROWS + 1];
  uint32_t n_complex;  // rows of this block that reached complexCompact in-wave
};

// Stages src[b0, b1) into lds with 16-B loads; byte x of src lands at
// lds[x - b0 + head], head = the misalignment of src + b0. Every loaded chunk
// holds at least one byte of the range, so no load leaves the range's pages.
DEVI uint32_t cq_stage(uint8_t* lds, const uint8_t* src, uint64_t b0, uint64_t b1, int tid) {
  const uintptr_t s = (uintptr_t)(src + b0);
  const uint32_t head = (uint32_t)(s & 15u);
  if (b1 <= b0) return head;
  const uint64_t nch = (head + (b1 - b0) + 15) / 16;
  const uint4* g = (const uint4*)(s - head);
  for (uint64_t c = tid; c < nch; c += 256) *(uint4*)(lds + 16 * c) = g[c];
  return head;
}

// Writes lds[i0 + (x - b0)] to dst[x] for x in [b0, b1): 16-B stores where a
// whole aligned chunk of dst lies inside the range, byte stores at the edges.
// lds must be laid out so that (i0 - (dst+b0)) is a multiple of 16.
DEVI void cq_unstage(uint8_t* dst, const uint8_t* lds, uint32_t i0, uint64_t b0, uint64_t b1, int tid) {
  if (b1 <= b0) return;
  const uintptr_t s = (uintptr_t)(dst + b0), e = (uintptr_t)(dst + b1);
  const uintptr_t a0 = s & ~(uintptr_t)15;
  const uint64_t nch = (e - a0 + 15) / 16;
  for (uint64_t c = tid; c < nch; c += 256) {
    const uintptr_t cs = a0 + 16 * c;
    const uint32_t li = (uint32_t)(i0 - (s - a0) + 16 * c);  // lds index of byte cs
    if (cs >= s && cs + 16 <= e) {
      *(uint4*)cs = *(const uint4*)(lds + li);
    } else {
      for (int j = 0; j < 16; j++)
        if (cs + j >= s && cs + j < e) *(uint8_t*)(cs + j) = lds[li + j];
    }
  }
}

DEVI uint32_t lds_q16(const uint8_t* p, uint32_t i) { return ((uint32_t)p[i] << 8) | p[i + 1]; }
DEVI uint32_t lds_u16(const uint8_t* p, uint32_t i) { return (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8); }

// Row positions inside the tile's LDS buffers.
struct RowLds {
  uint32_t k0;   // byte index of the row's first KV length in qlen
  uint32_t kv0;  // ... in vlen
  uint32_t qi;   // index of the row's first qualifier byte in qin
  uint32_t vi;   // ... first value byte in vin
  uint32_t qo;   // index in qout of the row's compacted qualifier
  uint32_t vo;   // index in vout of the row's compacted value
};

// Bitonic sort (ascending) of keys[0, n) by one wave; n <= CT_SORT.
DEVI void cq_sort(uint32_t* keys, uint32_t n, int lane) {
  uint32_t P = 2;
  while (P < n) P <<= 1;
  for (uint32_t i = n + lane; i < P; i += WAVE) keys[i] = ~0u;
  wave_lds_sync();
  for (uint32_t k = 2; k <= P; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = lane; i < P; i += WAVE) {
        const uint32_t l = i ^ j;
        if (l > i) {
          const uint32_t x = keys[i], y = keys[l];
          if ((x > y) == ((i & k) == 0)) {
            keys[i] = y;
            keys[l] = x;
          }
        }
      }
      wave_lds_sync();
    }
  }
}

// Number of keys in the sorted run A[rs, re) below `key` (keys are unique).
DEVI uint32_t cq_lower_bound(const uint32_t* A, uint32_t rs, uint32_t re, uint32_t key) {
  uint32_t lo = rs, hi = re;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (A[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo - rs;
}

constexpr int CQ_RUNS = 8;  // sorted runs merged by rank before falling back to bitonic

// complexCompact (:600-743) of one row from LDS. Returns the row status; on
// COMPLEX, *qlen/*vlen are the output lengths (already in qout/vout).
// The cells' stable sort order is the order of the composite key
// (qualifier << 16 | breakdown index). The 2-byte KVs that reach here have
// strictly increasing deltas (the trivial pre-pass threw otherwise), so they
// form one sorted run; each multi-value cell is a run when its qualifiers
// do not decrease (true for every cell trivialCompact/complexCompact wrote).
// With <= CQ_RUNS runs a cell's final position is the sum of its ranks in
// every run (binary searches); otherwise the keys are bitonic-sorted.
DEVI uint8_t cq_complex_lds(TileLds& L, const RowLds& p, uint32_t nk, uint32_t n_single, uint32_t n_cells,
                            uint32_t* A, uint32_t* pay, uint32_t* runs, int lane, uint32_t* qlen_out,
                            uint32_t* vlen_out) {
  // ---- breakDownValues: singles at A[0, n_single), multi cells after ----
  uint32_t qcar = 0, vcar = 0, ccar = 0, scar = 0, mcar = n_single;
  uint32_t err = ~0u;  // (kv << 1) | oob of the first failing KV
  uint32_t nruns = n_single ? 1u : 0u;
  bool monotone = true;
  if (lane == 0) runs[0] = 0;
  for (uint32_t base = 0; base < nk; base += WAVE) {
    const uint32_t i = base + lane;
    const bool act = i < nk;
    const uint32_t ql = act ? lds_u16(L.qlen, p.k0 + 2 * i) : 0u;
    const uint32_t vl = act ? lds_u16(L.vlen, p.kv0 + 2 * i) : 0u;
    const bool valid = act && ql != 0 && (ql & 1) == 0;
    const bool two = valid && ql == 2;
    const uint32_t nc = valid ? ql >> 1 : 0u;
    const uint32_t qx = wave_incl_scan_u32_dpp(ql), vx = wave_incl_scan_u32_dpp(vl), cx = wave_incl_scan_u32_dpp(nc);
    const uint32_t qpos = p.qi + qcar + qx - ql, vpos = p.vi + vcar + vx - vl, cb = ccar + cx - nc;
    qcar += readlane_u32(qx, 63);
    vcar += readlane_u32(vx, 63);
    ccar += readlane_u32(cx, 63);
    const uint64_t m2 = ballot(two);
    if (two) {
      const uint32_t q = lds_q16(L.qin, qpos);
      const bool leg = cq_legacy(q & 0xFF, vl);
      const uint32_t flen = leg ? 4u : vl;
      A[scar + __popcll(m2 & lanemask_lt(lane))] = (((q & 0xFF00) | cq_fixq(q & 0xFF, flen)) << 16) | cb;
      pay[cb] = ((vpos + (leg ? 4u : 0u)) << 16) | flen;
    }
    const bool bad = two && cq_legacy(lds_q16(L.qin, qpos) & 0xFF, vl) &&
                     (L.vin[vpos] | L.vin[vpos + 1] | L.vin[vpos + 2] | L.vin[vpos + 3]) != 0;
    const uint64_t mb = ballot(bad);
    if (mb) err = min(err, (base + (uint32_t)(__ffsll((long long)mb) - 1)) << 1);
    scar += __popcll(m2);
    uint64_t mm = ballot(valid && ql > 2);
    while (mm) {  // multi-value cells, one at a time, wave-cooperative
      const int l = __ffsll((long long)mm) - 1;
      mm &= mm - 1;
      const uint32_t kq = readlane_u32(qpos, l), kv = readlane_u32(vpos, l);
      const uint32_t kvl = readlane_u32(vl, l), knc = readlane_u32(nc, l), kcb = readlane_u32(cb, l);
      const uint32_t kid = base + l;
      if (nruns < CQ_RUNS && lane == 0) runs[nruns] = mcar;
      nruns++;
      if (kvl == 0) {  // val[val.length - 1] of an empty value (:708)
        err = min(err, (kid << 1) | 1u);
        continue;
      }
      if (L.vin[kv + kvl - 1] != 0) {  // unknown meta byte (:709-714)
        err = min(err, kid << 1);
        continue;
      }
      uint32_t run = 0, prevq = 0;
      bool over = false, desc = false;
      for (uint32_t c0 = 0; c0 < knc; c0 += WAVE) {
        const uint32_t c = c0 + lane;
        const bool a2 = c < knc;
        const uint32_t q = a2 ? lds_q16(L.qin, kq + 2 * c) : 0u;
        const uint32_t len = a2 ? (q & 7u) + 1u : 0u;
        const uint32_t incl = wave_incl_scan_u32_dpp(len);
        const uint32_t off = run + incl - len;
        uint32_t pq = (uint32_t)__shfl((int)q, lane == 0 ? 0 : lane - 1);
        if (lane == 0) pq = prevq;
        if (a2) {
          over |= off + len > kvl;  // System.arraycopy past the value (:722)
          desc |= q < pq;
          A[mcar + c] = (q << 16) | (kcb + c);
          pay[kcb + c] = ((kv + off) << 16) | len;
        }
        run += readlane_u32(incl, 63);
        prevq = (uint32_t)__shfl((int)q, 63);
      }
      monotone = monotone && !ballot(desc);
      mcar += knc;
      if (ballot(over)) err = min(err, (kid << 1) | 1u);
      else if (run != kvl - 1) err = min(err, kid << 1);  // (:730-736)
    }
  }
  if (err != ~0u) return (err & 1u) ? CQ_OOB : CQ_ERROR;
  const uint32_t n = n_cells;
  wave_lds_sync();
  if (monotone && nruns <= CQ_RUNS) {
    // ---- merge the sorted runs by rank ----
    if (lane == 0) runs[nruns] = n;
    wave_lds_sync();
    uint32_t key[CT_SORT / WAVE], rank[CT_SORT / WAVE];
#pragma unroll
    for (int k = 0; k < CT_SORT / WAVE; k++) {
      const uint32_t i = lane + WAVE * k;
      key[k] = i < n ? A[i] : 0u;
      rank[k] = 0;
      if (i < n) {
        for (uint32_t r = 0; r < nruns; r++) {
          const uint32_t rs = runs[r], re = runs[r + 1];
          rank[k] += (i >= rs && i < re) ? i - rs : cq_lower_bound(A, rs, re, key[k]);
        }
      }
    }
    wave_lds_sync();
#pragma unroll
    for (int k = 0; k < CT_SORT / WAVE; k++)
      if (lane + WAVE * k < n) A[rank[k]] = key[k];
    wave_lds_sync();
  } else {
    cq_sort(A, n, lane);
  }
  // ---- duplicate check + emission in sorted order (:611-678) ----
  int prev_d = -1;
  uint32_t rep_key = 0, rank = 0, vrun = 0;
  bool bad = false;
  for (uint32_t p0 = 0; p0 < n; p0 += WAVE) {
    const uint32_t i = p0 + lane;
    const bool act = i < n;
    const uint32_t key = act ? A[i] : ~0u;
    const int d = (int)(key >> 20);
    int pd = __shfl(d, lane == 0 ? 0 : lane - 1);
    if (lane == 0) pd = prev_d;
    const bool head = act && d != pd;
    const uint64_t hm = ballot(head);
    const uint64_t below = hm & lanemask_le(lane);
    const uint32_t sk = (uint32_t)__shfl((int)key, below ? 63 - __clzll(below) : lane);
    const uint32_t rk = below ? sk : rep_key;
    const uint32_t pw = act ? pay[key & 0xFFFF] : 0u;
    const uint32_t len = pw & 0xFFFF, off = pw >> 16;
    if (act && !head) {
      const uint32_t rw = pay[rk & 0xFFFF];
      if (((key >> 16) & 0xFF) != ((rk >> 16) & 0xFF) || len != (rw & 0xFFFF)) {
        bad = true;
      } else {
        for (uint32_t j = 0; j < len; j++) bad |= L.vin[off + j] != L.vin[(rw >> 16) + j];
      }
    }
    const uint32_t hl = head ? len : 0u;
    const uint32_t vi = wave_incl_scan_u32_dpp(hl);
    if (head) {
      const uint32_t r2 = rank + __popcll(hm & lanemask_lt(lane));
      L.qout[p.qo + 2 * r2] = (uint8_t)(key >> 24);
      L.qout[p.qo + 2 * r2 + 1] = (uint8_t)(key >> 16);
      const uint32_t dst = p.vo + vrun + vi - hl;
      for (uint32_t j = 0; j < len; j++) L.vout[dst + j] = L.vin[off + j];
    }
    rank += __popcll(hm);
    vrun += readlane_u32(vi, 63);
    prev_d = __shfl(d, 63);
    if (hm) rep_key = (uint32_t)__shfl((int)key, 63 - __clzll(hm));
  }
  if (ballot(bad)) return CQ_ERROR;
  if (lane == 0) L.vout[p.vo + vrun] = 0;
  *qlen_out = 2 * rank;
  *vlen_out = vrun + 1;
  return CQ_COMPLEX;
}

// One row, LDS -> LDS (same classification as cq_row_global). Returns false
// when the row went to the block kernels (complexCompact of > CT_SORT cells).
DEVI bool cq_row_lds(const CompactArgs& a, uint64_t r, const RowHdr& h, TileLds& L, const RowLds& p,
                     uint32_t* keys, uint32_t* pay, uint32_t* runs, int lane, uint32_t* qlen_out = nullptr,
                     uint32_t* vlen_out = nullptr) {
  const uint32_t nk = (uint32_t)h.nk;
  uint32_t qcar = 0, vcar = 0, nvalid = 0, nmulti = 0, ncells = 0;
  int last_delta = -1;
  bool err_delta = false, legacy_bad = false, any_fix = false, any_junk = false;
  uint32_t f_qpos = 0, f_vpos = 0, f_ql = 0, f_vl = 0, f_q = 0;
  for (uint32_t base = 0; base < nk; base += WAVE) {
    const uint32_t i = base + lane;
    const bool act = i < nk;
    const uint32_t ql = act ? lds_u16(L.qlen, p.k0 + 2 * i) : 0u;
    const uint32_t vl = act ? lds_u16(L.vlen, p.kv0 + 2 * i) : 0u;
    const uint32_t qi = wave_incl_scan_u32_dpp(ql), vi = wave_incl_scan_u32_dpp(vl);
    // (clamped: lengths that overrun the row are rejected after this pass)
    const uint32_t qpos = min(p.qi + qcar + qi - ql, (uint32_t)CT_QB), vpos = min(p.vi + vcar + vi - vl, (uint32_t)CT_VB);
    qcar += readlane_u32(qi, 63);
    vcar += readlane_u32(vi, 63);
    const bool valid = act && ql != 0 && (ql & 1) == 0;
    const bool two = valid && ql == 2;
    const uint32_t q = two ? lds_q16(L.qin, qpos) : 0u;
    const int delta = (int)(q >> 4);
    const bool leg = two && cq_legacy(q & 0xFF, vl);
    const bool lbad = leg && (L.vin[vpos] | L.vin[vpos + 1] | L.vin[vpos + 2] | L.vin[vpos + 3]) != 0;
    const uint64_t m2 = ballot(two);
    const uint64_t lower = m2 & lanemask_lt(lane);
    int pd = __shfl(delta, lower ? 63 - __clzll(lower) : lane);
    if (!lower) pd = last_delta;
    err_delta |= ballot(two && delta <= pd) != 0;
    if (m2) last_delta = __shfl(delta, 63 - __clzll(m2));
    legacy_bad |= ballot(lbad) != 0;
    // a KV whose bytes change in trivialCompact: legacy float or wrong length flags
    any_fix |= ballot(two && (leg || cq_fixq(q & 0xFF, vl) != (q & 0xFF))) != 0;
    any_junk |= ballot(act && !valid) != 0;
    const uint64_t mv = ballot(valid);
    if (nvalid == 0 && mv) {
      const int fl = __ffsll((long long)mv) - 1;
      f_qpos = readlane_u32(qpos, fl);
      f_vpos = readlane_u32(vpos, fl);
      f_ql = readlane_u32(ql, fl);
      f_vl = readlane_u32(vl, fl);
      f_q = readlane_u32(q, fl);
    }
    nvalid += __popcll(mv);
    nmulti += __popcll(ballot(valid && ql > 2));
    ncells += readlane_u32(wave_incl_scan_u32_dpp(valid ? ql >> 1 : 0u), 63);
  }
  uint8_t st;
  uint32_t oql = 0, ovl = 0;
  if (qcar != h.qe - h.qs || vcar != h.ve - h.vs) {  // lengths vs extents: E_INVALID_ARG
    if (lane == 0) atomicOr(&a.counters[2], 1u);
    st = CQ_NONE;
  } else if (nvalid == 0) {
    st = CQ_NONE;
  } else if (nvalid == 1) {
    if (f_ql == 2 && cq_legacy(f_q & 0xFF, f_vl)) {
      if ((L.vin[f_vpos] | L.vin[f_vpos + 1] | L.vin[f_vpos + 2] | L.vin[f_vpos + 3]) != 0) {
        st = CQ_ERROR;
      } else {
        st = CQ_SINGLE;
        if (lane < 4) L.vout[p.vo + lane] = L.vin[f_vpos + 4 + lane];
        if (lane == 0) {
          L.qout[p.qo] = (uint8_t)(f_q >> 8);
          L.qout[p.qo + 1] = (uint8_t)cq_fixq(f_q & 0xFF, 4);
        }
        oql = 2;
        ovl = 4;
      }
    } else {
      st = CQ_SINGLE;
      for (uint32_t j = lane; j < f_ql; j += WAVE) L.qout[p.qo + j] = L.qin[f_qpos + j];
      for (uint32_t j = lane; j < f_vl; j += WAVE) L.vout[p.vo + j] = L.vin[f_vpos + j];
      oql = f_ql;
      ovl = f_vl;
    }
  } else if (err_delta || (nmulti == 0 && legacy_bad)) {
    st = CQ_ERROR;
  } else if (nmulti) {
    if (ncells <= CT_SORT) {
      st = cq_complex_lds(L, p, nk, nvalid - nmulti, ncells, keys, pay, runs, lane, &oql, &ovl);
      if (lane == 0) atomicAdd(&L.n_complex, 1u);
    } else {  // too many cells for the in-wave sort: block kernels
      if (lane == 0) {
        if (ncells <= CQ_LDS_CELLS) a.list_lds[atomicAdd(&a.counters[0], 1u)] = (uint32_t)r;
        else a.list_big[atomicAdd(&a.counters[1], 1u)] = (uint32_t)r;
      }
      return false;
    }
  } else if (!any_fix && !any_junk) {
    // trivialCompact changes nothing: qualifiers and values pass through
    st = CQ_TRIVIAL;
    for (uint32_t j = lane; j < qcar; j += WAVE) L.qout[p.qo + j] = L.qin[p.qi + j];
    for (uint32_t j = lane; j < vcar; j += WAVE) L.vout[p.vo + j] = L.vin[p.vi + j];
    if (lane == 0) L.vout[p.vo + vcar] = 0;
    oql = qcar;
    ovl = vcar + 1;
  } else {
    // trivialCompact (:450-474) with flag / legacy-float fixes and junk skipped
    st = CQ_TRIVIAL;
    uint32_t qc2 = 0, vc2 = 0, nq = 0, nv = 0;
    for (uint32_t base = 0; base < nk; base += WAVE) {
      const uint32_t i = base + lane;
      const bool act = i < nk;
      const uint32_t ql = act ? lds_u16(L.qlen, p.k0 + 2 * i) : 0u;
      const uint32_t vl = act ? lds_u16(L.vlen, p.kv0 + 2 * i) : 0u;
      const uint32_t qi = wave_incl_scan_u32_dpp(ql), vi = wave_incl_scan_u32_dpp(vl);
      const uint32_t qpos = p.qi + qc2 + qi - ql, vpos = p.vi + vc2 + vi - vl;
      qc2 += readlane_u32(qi, 63);
      vc2 += readlane_u32(vi, 63);
      const bool valid = act && ql == 2;
      const uint32_t q = valid ? lds_q16(L.qin, qpos) : 0u;
      const bool leg = valid && cq_legacy(q & 0xFF, vl);
      const uint32_t flen = valid ? (leg ? 4u : vl) : 0u;
      const uint64_t mv = ballot(valid);
      const uint32_t fi = wave_incl_scan_u32_dpp(flen);
      if (valid) {
        const uint32_t o = p.qo + 2 * (nq + __popcll(mv & lanemask_lt(lane)));
        L.qout[o] = (uint8_t)(q >> 8);
        L.qout[o + 1] = (uint8_t)cq_fixq(q & 0xFF, flen);
        const uint32_t src = vpos + (leg ? 4u : 0u), dst = p.vo + nv + fi - flen;
        for (uint32_t j = 0; j < flen; j++) L.vout[dst + j] = L.vin[src + j];
      }
      nq += __popcll(mv);
      nv += readlane_u32(fi, 63);
    }
    if (lane == 0) L.vout[p.vo + nv] = 0;
    oql = 2 * nq;
    ovl = nv + 1;
  }
  if (lane == 0) cq_finish(a, r, st, oql, ovl);
  if (qlen_out) {
    *qlen_out = oql;
    *vlen_out = ovl;
  }
  return true;
}

__global__ void __launch_bounds__(256) k_compact_tiles(CompactArgs a) {
  __shared__ TileLds L;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
  const uint64_t n_tiles = (a.n_rows + CT_ROWS - 1) / CT_ROWS;
  const uint64_t Q0 = a.row_qual_off[0], V0 = a.row_val_off[0];
  if (tid == 0) L.n_complex = 0;
  for (uint64_t t = blockIdx.x; t < n_tiles; t += gridDim.x) {
    const uint64_t r0 = t * CT_ROWS;
    const uint32_t nr = (uint32_t)min((uint64_t)CT_ROWS, a.n_rows - r0);
    __syncthreads();  // previous tile's LDS fully consumed
    if (tid <= (int)nr) {
      L.hdr[0][tid] = a.row_kv_start[r0 + tid];
      L.hdr[1][tid] = a.row_qual_off[r0 + tid];
      L.hdr[2][tid] = a.row_val_off[r0 + tid];
    }
    __syncthreads();
    const uint64_t kb0 = L.hdr[0][0], kb1 = L.hdr[0][nr];
    const uint64_t qs0 = L.hdr[1][0], qs1 = L.hdr[1][nr];
    const uint64_t vs0 = L.hdr[2][0], vs1 = L.hdr[2][nr];
    const bool fits = kb0 <= kb1 && kb1 <= a.n_kvs && kb1 - kb0 <= CT_KB && qs0 <= qs1 && qs1 <= a.qual_nbytes &&
                      qs1 - qs0 <= CT_QB && vs0 <= vs1 && vs1 <= a.val_nbytes && vs1 - vs0 <= CT_VB &&
                      qs0 >= Q0 && vs0 >= V0 && qs1 - Q0 <= a.qcap && vs1 - V0 + r0 + nr <= a.vcap;
    if (!fits) {
      for (uint32_t j = w; j < nr; j += 4) cq_row_global(a, r0 + j, lane);
      continue;
    }
    // ---- stage the tile (one round trip) ----
    const uint32_t hq = cq_stage(L.qin, a.qual, qs0, qs1, tid);
    const uint32_t hv = cq_stage(L.vin, a.val, vs0, vs1, tid);
    const uint32_t hk = cq_stage(L.qlen, (const uint8_t*)a.kv_qual_len, 2 * kb0, 2 * kb1, tid);
    const uint32_t hkv = cq_stage(L.vlen, (const uint8_t*)a.kv_val_len, 2 * kb0, 2 * kb1, tid);
    // output buffers share the destination's 16-B phase (for cq_unstage)
    const uint32_t oq_h = (uint32_t)((uintptr_t)(a.oq + (qs0 - Q0)) & 15u);
    const uint32_t ov_h = (uint32_t)((uintptr_t)(a.ov + (vs0 - V0 + r0)) & 15u);
    __syncthreads();
    for (uint32_t j = w; j < nr; j += 4) {
      const uint64_t r = r0 + j;
      RowHdr h;
      h.kb = L.hdr[0][j];
      h.nk = L.hdr[0][j + 1] - h.kb;
      h.qs = L.hdr[1][j];
      h.qe = L.hdr[1][j + 1];
      h.vs = L.hdr[2][j];
      h.ve = L.hdr[2][j + 1];
      h.oqo = h.qs - Q0;
      h.ovo = h.vs - V0 + r;
      if (lane == 0) {
        a.out_qoff[r] = h.oqo;
        a.out_voff[r] = h.ovo;
      }
      // offsets must not decrease (else E_INVALID_ARG); the lengths are
      // checked against the extents in cq_row_lds
      if (!(L.hdr[0][j + 1] >= h.kb && h.qe >= h.qs && h.ve >= h.vs)) {
        if (lane == 0) {
          atomicOr(&a.counters[2], 1u);
          cq_finish(a, r, CQ_NONE, 0, 0);
        }
        continue;
      }
      RowLds p;
      p.k0 = hk + 2 * (uint32_t)(h.kb - kb0);
      p.kv0 = hkv + 2 * (uint32_t)(h.kb - kb0);
      p.qi = hq + (uint32_t)(h.qs - qs0);
      p.vi = hv + (uint32_t)(h.vs - vs0);
      p.qo = oq_h + (uint32_t)(h.qs - qs0);
      p.vo = ov_h + (uint32_t)(h.vs - vs0) + j;
      cq_row_lds(a, r, h, L, p, L.keys[w], L.pay[w], L.runs[w], lane);
    }
    __syncthreads();
    // ---- write the tile's compacted bytes back ----
    cq_unstage(a.oq, L.qout, oq_h, qs0 - Q0, qs1 - Q0, tid);
    cq_unstage(a.ov, L.vout, ov_h, vs0 - V0 + r0, vs1 - V0 + r0 + nr, tid);
  }
  __syncthreads();
  if (tid == 0 && L.n_complex) atomicAdd(&a.counters[3], L.n_complex);
}

// ===========================================================================
// k_compact_dups: the write/delete decision of complexCompact rows
// (CompactionQueue.java:355-404). `longest` is the row's first KV as handed
// in, replaced by each later non-2-byte, even, non-empty qualifier strictly
// longer than it (:283-312); if the compacted qualifier is not longer than
// longest's, the KV holding exactly the compacted qualifier — longest itself
// if it matches, else the first such KV in row order (:369-387) — is kept
// out of the delete set, and nothing is written when its value is the
// compacted value too (:388-399). One wave per row, only for COMPLEX rows
// (found by a ballot over 64 rows' statuses); reads the row's KV lengths and
// the candidate qualifiers again, and the compacted bytes just written.
// ===========================================================================
DEVI bool cq_wave_equal(const uint8_t* x, const uint8_t* y, uint32_t n, int lane) {
  bool ne = false;
  for (uint32_t j = lane; j < n; j += WAVE) ne |= x[j] != y[j];
  return ballot(ne) == 0;
}

DEVI void cq_dup_row(const CompactArgs& a, uint64_t r, int lane) {
  const uint64_t kb = a.row_kv_start[r], nk = a.row_kv_start[r + 1] - kb;
  const uint64_t qs = a.row_qual_off[r], vs = a.row_val_off[r];
  const uint32_t cql = a.out_qlen[r], cvl = a.out_vlen[r];
  const uint8_t* cq = a.oq + a.out_qoff[r];
  const uint8_t* cv = a.ov + a.out_voff[r];
  // ---- longest (:283-312) ----
  uint32_t lbest = a.kv_qual_len[kb];
  uint64_t li = 0, lq = qs, lv = vs;
  uint32_t lvl = a.kv_val_len[kb];
  uint64_t qcar = 0, vcar = 0;
  for (uint64_t base = 0; base < nk; base += WAVE) {
    const uint64_t i = base + lane;
    const bool act = i < nk;
    const uint32_t ql = act ? a.kv_qual_len[kb + i] : 0u, vl = act ? a.kv_val_len[kb + i] : 0u;
    const uint32_t qi = wave_incl_scan_u32_dpp(ql), vi = wave_incl_scan_u32_dpp(vl);
    const uint64_t qpos = qs + qcar + (qi - ql), vpos = vs + vcar + (vi - vl);
    qcar += readlane_u32(qi, 63);
    vcar += readlane_u32(vi, 63);
    const bool multi = act && ql != 2 && ql != 0 && (ql & 1) == 0;
    uint32_t mx = multi ? ql : 0u;
#pragma unroll
    for (int m = 1; m < WAVE; m <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, m));
    if (mx > lbest) {  // first KV of this chunk at the new maximum
      const int fl = __ffsll((long long)ballot(multi && ql == mx)) - 1;
      lbest = mx;
      li = base + fl;
      lq = readlane_u64(qpos, fl);
      lv = readlane_u64(vpos, fl);
      lvl = readlane_u32(vl, fl);
    }
  }
  if (cql > lbest) return;  // :366 — cannot overwrite an existing cell
  // ---- the KV holding the compacted qualifier (:369-387) ----
  int64_t dup = -1;
  uint64_t dvpos = 0;
  uint32_t dvl = 0;
  if (lbest == cql && cq_wave_equal(a.qual + lq, cq, cql, lane)) {
    dup = (int64_t)li;
    dvpos = lv;
    dvl = lvl;
  } else {
    qcar = vcar = 0;
    for (uint64_t base = 0; base < nk && dup < 0; base += WAVE) {
      const uint64_t i = base + lane;
      const bool act = i < nk;
      const uint32_t ql = act ? a.kv_qual_len[kb + i] : 0u, vl = act ? a.kv_val_len[kb + i] : 0u;
      const uint32_t qi = wave_incl_scan_u32_dpp(ql), vi = wave_incl_scan_u32_dpp(vl);
      const uint64_t qpos = qs + qcar + (qi - ql), vpos = vs + vcar + (vi - vl);
      qcar += readlane_u32(qi, 63);
      vcar += readlane_u32(vi, 63);
      uint64_t cand = ballot(act && ql == cql);
      while (cand) {
        const int l = __ffsll((long long)cand) - 1;
        cand &= cand - 1;
        if (cq_wave_equal(a.qual + readlane_u64(qpos, l), cq, cql, lane)) {
          dup = (int64_t)(base + l);
          dvpos = readlane_u64(vpos, l);
          dvl = readlane_u32(vl, l);
          break;
        }
      }
    }
  }
  if (dup < 0) return;
  const bool same = dvl == cvl && cq_wave_equal(a.val + dvpos, cv, cvl, lane);  // :391
  if (lane == 0) {
    if (same) a.out_write[r] = 0;
    a.out_keep[r] = (int32_t)dup;  // :399
  }
}

__global__ void __launch_bounds__(256) k_compact_dups(CompactArgs a) {
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + threadIdx.x / WAVE; g * WAVE < a.n_rows; g += nw) {
    const uint64_t r = g * WAVE + lane;
    uint64_t m = ballot(r < a.n_rows && a.status[r] == CQ_COMPLEX);
    while (m) {
      const int l = __ffsll((long long)m) - 1;
      m &= m - 1;
      cq_dup_row(a, g * WAVE + l, lane);
    }
  }
}

// ===========================================================================
// The plain-row path. A row is plain when it holds >= 2 KVs, every qualifier
// is 2 bytes, every value has 1..8 bytes, legacy floats are fixable and the
// time deltas strictly increase in KV order: trivialCompact's output is then
// the row's qualifier and value bytes with two local fix-ups, plus the 0 meta
// byte (CompactionQueue.java:286-351, 450-474, fixes :490-544):
//   * fixQualifierFlags: a qualifier's length bits become the fixed value's
//     length - 1 (one byte patched in place);
//   * fixFloatingPointValue: a legacy float's 8-byte value 00000000 || bits
//     loses its 4-byte zero prefix (the row's later value bytes move down).
// With the output placement of tsdbhip.h the qualifier stream is copied in
// place and the value stream shifted by one byte per row. Four launches:
//   k_compact_quals     the qualifier bytes, in place, 16-B stores
//   k_compact_classify  one row per 16-lane quarter wave: the plain test;
//                       flag fix-ups patched over the copied qualifiers; the
//                       holes (output positions of the first two legacy
//                       floats) recorded; plain rows get status / lengths /
//                       write decision, the others CQ_PENDING
//   k_compact_vals      the value bytes around the holes, 16-B stores
//   k_compact_rows      the CQ_PENDING rows (gathered per 256-row range)
//                       through the LDS row logic of k_compact_tiles
// ===========================================================================
constexpr uint32_t CC_ROWS = 64;  // rows per copy tile (one block)
#ifndef CP_U
#define CP_U 2  // KV batches of 16 per row whose loads are in flight together (4: 0.329 ms, 3: 0.320, 2: 0.286 on C5)
#endif

// Inclusive scan inside each 16-lane DPP row (= one quarter of the wave).
DEVI uint32_t quarter_incl_scan_u32(uint32_t x) {
  x += dpp_u32<0x111, 0xf>(x);
  x += dpp_u32<0x112, 0xf>(x);
  x += dpp_u32<0x114, 0xf>(x);
  x += dpp_u32<0x118, 0xf>(x);
  return x;
}
// lane l gets lane l-1's x inside its quarter; a quarter's lane 0 gets `old`
DEVI uint32_t quarter_shr1_u32(uint32_t x, uint32_t old) {
  return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, 0x111, 0xf, 0xf, false);
}

// Runs after k_compact_quals. One row per 16-lane quarter of a wave, its KVs
// 16 x CP_U at a time (every load of a batch in flight together). Qualifier
// fix-ups are written while the row's later KVs are still unseen: a row that
// turns out not plain gets them too, inside its own output range, where
// k_compact_rows then writes its real result.
__global__ void __launch_bounds__(256) k_compact_classify(CompactArgs a) {
  const int lane = lane_id(), sub = lane & 15, qtr = lane >> 4;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  const uint64_t Q0 = a.row_qual_off[0], V0 = a.row_val_off[0];
  const uint64_t n_quads = (a.n_rows + 3) / 4;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + threadIdx.x / WAVE; g < n_quads; g += nw) {
    const uint64_t r = 4 * g + qtr;
    const bool own = r < a.n_rows;
    uint64_t kv = 0, kv_n = 0, qo = 0, qo_n = 0, vo = 0, vo_n = 0;
    if (own) {
      kv = a.row_kv_start[r];
      kv_n = a.row_kv_start[r + 1];
      qo = a.row_qual_off[r];
      qo_n = a.row_qual_off[r + 1];
      vo = a.row_val_off[r];
      vo_n = a.row_val_off[r + 1];
    }
    // the row's own output ranges, when its offsets are sane (disjoint from
    // every other row's then)
    const bool sane = own && kv_n >= kv && kv_n <= a.n_kvs && qo_n >= qo && vo_n >= vo && qo >= Q0 && vo >= V0 &&
                      qo_n <= a.qual_nbytes && vo_n <= a.val_nbytes && qo_n - Q0 <= a.qcap &&
                      vo_n - V0 + r + 1 <= a.vcap && vo_n - vo < (1ull << 32);
    const uint64_t nk = sane ? kv_n - kv : 0;
    bool plain = sane && nk >= 2 && qo_n - qo == 2 * nk;
    const uint64_t nkw = plain ? nk : 0;  // KVs walked
    const uint64_t ovo = vo - V0 + r;
    uint32_t vcar = 0, legs = 0, q_prev = 0;  // (uniform per quarter)
    uint32_t h0 = ~0u, h1 = ~0u;  // output positions of the row's holes (legacy floats)
    bool bad = false;
    for (uint64_t i0 = 0; ballot(i0 < nkw); i0 += 16 * CP_U) {
      uint32_t ql_[CP_U], vl_[CP_U], q_[CP_U];
#pragma unroll
      for (int u = 0; u < CP_U; u++) {
        const uint64_t i = i0 + 16 * u + sub;
        ql_[u] = vl_[u] = q_[u] = 0;
        if (i < nkw) {
          ql_[u] = a.kv_qual_len[kv + i];
          vl_[u] = a.kv_val_len[kv + i];
          q_[u] = ld_q16(a.qual, qo + 2 * i);  // (the qualifier if every one has 2 bytes)
        }
      }
      uint32_t voff_[CP_U], fl_[CP_U];  // fl: 1 bad, 2 legacy, nleg << 2
#pragma unroll
      for (int u = 0; u < CP_U; u++) {
        const uint64_t i = i0 + 16 * u + sub;
        const bool act = i < nkw;
        const uint32_t ql = ql_[u], vl = vl_[u], q = q_[u];
        bool kbad = act && (ql != 2 || vl == 0 || vl > 8);
        const bool legacy = act && !kbad && cq_legacy(q & 0xFFu, vl);  // floatingPointValueToFix :510-515
        const uint32_t incl = quarter_incl_scan_u32(act ? vl : 0u);
        const uint32_t vin = vcar + incl - (act ? vl : 0u);  // value offset inside the row
        const uint64_t lm = (ballot(legacy) >> (16 * qtr)) & 0xFFFFu;
        const uint32_t nleg = legs + (uint32_t)__popcll(lm & ((1u << sub) - 1));
        const uint32_t qb = quarter_shr1_u32(q, q_prev);
        if (act && !kbad) kbad = (uint64_t)vin + vl > vo_n - vo || (i > 0 && (q >> 4) <= (qb >> 4));
        voff_[u] = vin;
        fl_[u] = (kbad ? 1u : 0u) | (legacy ? 2u : 0u);
        if (ballot(legacy)) {  // the holes: output positions of the first two legacy floats
          const uint32_t P = vin - 4 * nleg;
          const uint32_t f0 = (uint32_t)__builtin_ctz((uint32_t)lm | 0x10000u);
          const uint32_t lm1 = (uint32_t)lm & ((uint32_t)lm - 1);
          const uint32_t f1 = (uint32_t)__builtin_ctz(lm1 | 0x10000u);
          const uint32_t p0 = (uint32_t)__shfl((int)P, (lane & 48) | (int)(f0 & 15));
          const uint32_t p1 = (uint32_t)__shfl((int)P, (lane & 48) | (int)(f1 & 15));
          if (lm) {
            if (legs == 0) {
              h0 = p0;
              if (lm1) h1 = p1;
            } else if (legs == 1) {
              h1 = p0;
            }
          }
        }
        vcar += (uint32_t)__shfl((int)incl, lane | 15);
        legs += (uint32_t)__popcll(lm);
        q_prev = (uint32_t)__shfl((int)q, lane | 15);
      }
      // legacy floats: the 4-byte zero prefix (fixFloatingPointValue :530-544)
      uint32_t pre_[CP_U];
#pragma unroll
      for (int u = 0; u < CP_U; u++) {
        pre_[u] = 0;
        if ((fl_[u] & 3u) == 2u) {
          const uint64_t vf = vo + voff_[u];
          pre_[u] = a.val[vf] | a.val[vf + 1] | a.val[vf + 2] | a.val[vf + 3];
        }
      }
      // the qualifier fix-ups (speculatively), rows with a bad KV
#pragma unroll
      for (int u = 0; u < CP_U; u++) {
        const uint64_t i = i0 + 16 * u + sub;
        const bool act = i < nkw;
        const bool legacy = (fl_[u] & 2u) != 0;
        const bool kbad = act && ((fl_[u] & 1u) || pre_[u] != 0);
        if (act && !kbad) {
          const uint32_t q = q_[u];
          const uint8_t f = (uint8_t)cq_fixq(q & 0xFFu, legacy ? 4u : vl_[u]);  // fixQualifierFlags :490-499
          if (f != (uint8_t)q) a.oq[qo - Q0 + 2 * i + 1] = f;
        }
        if ((ballot(kbad) >> (16 * qtr)) & 0xFFFFu) bad = true;
      }
    }
    if (plain) plain = !bad && legs <= 2 && vcar == vo_n - vo && !a.tile_bad[r / CC_ROWS];
    if (sub == 0 && plain) {
      const uint64_t vx = vo_n - vo;
      a.out_qoff[r] = qo - Q0;
      a.out_voff[r] = ovo;
      a.row_holes[r] = make_uint2(h0, h1);
      cq_finish(a, r, CQ_TRIVIAL, (uint32_t)(qo_n - qo), (uint32_t)(vx - 4ull * legs + 1));
    }
    if (sub == 0 && own && !plain) {
      a.status[r] = CQ_PENDING;  // (to the LDS row kernel)
      a.row_holes[r] = make_uint2(~0u, ~0u);
    }
  }
}

// 16 bytes at src + x (any alignment) from two aligned 16-B loads (the
// buffers carry >= 16 bytes of slack past their ends).
DEVI uint4 ld16_any(const uint8_t* src, uint64_t x) {
  const uintptr_t pa = (uintptr_t)(src + x);
  const uint4* p = (const uint4*)(pa & ~(uintptr_t)15);
  const uint32_t sh = (uint32_t)(pa & 15);
  const uint4 A = p[0];
  const uint4 B = p[1];  // (also when aligned: no branch; alignbyte by 0 keeps A)
  const uint32_t w[8] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w};
  const uint32_t s4 = sh >> 2, sb = sh & 3;
  uint32_t v[5];
#pragma unroll
  for (int i = 0; i < 5; i++) v[i] = s4 == 0 ? w[i] : s4 == 1 ? w[i + 1] : s4 == 2 ? w[i + 2] : w[i + 3];
  return make_uint4(__builtin_amdgcn_alignbyte(v[1], v[0], sb), __builtin_amdgcn_alignbyte(v[2], v[1], sb),
                    __builtin_amdgcn_alignbyte(v[3], v[2], sb), __builtin_amdgcn_alignbyte(v[4], v[3], sb));
}

// Select of two 16-byte vectors: bytes [0, p) from A, byte p = 0 when zp,
// the rest from B (p in [0, 16]).
DEVI uint4 cq_funnel(const uint4& A, const uint4& B, int p, bool zp) {
  const uint32_t av[4] = {A.x, A.y, A.z, A.w}, bv[4] = {B.x, B.y, B.z, B.w};
  uint32_t ov[4];
#pragma unroll
  for (int w = 0; w < 4; w++) {
    const int d = p - 4 * w;  // p's index inside dword w
    const uint32_t mA = d >= 4 ? ~0u : d <= 0 ? 0u : (1u << (8 * d)) - 1;
    const uint32_t mZ = (zp && d >= 0 && d < 4) ? 0xFFu << (8 * d) : 0u;
    ov[w] = (av[w] & mA) | (bv[w] & ~(mA | mZ));
  }
  return make_uint4(ov[0], ov[1], ov[2], ov[3]);
}

// Qualifiers of a tile of CC_ROWS rows copied in place (16-B stores, byte
// stores only at the tile's two edges); tiles with offsets out of bounds are
// flagged in tile_bad and left to the row kernel.
__global__ void __launch_bounds__(256) k_compact_quals(CompactArgs a) {
  const int tid = threadIdx.x;
  const uint64_t Q0 = a.row_qual_off[0];
  const uintptr_t oq_abs = (uintptr_t)a.oq;
  for (uint64_t t = blockIdx.x; t * CC_ROWS < a.n_rows; t += gridDim.x) {
    const uint64_t r0 = t * CC_ROWS;
    const uint32_t nr = (uint32_t)min((uint64_t)CC_ROWS, a.n_rows - r0);
    const uint64_t qa = a.row_qual_off[r0], qb = a.row_qual_off[r0 + nr];
    const bool skip = qa < Q0 || qb < qa || qb > a.qual_nbytes || qb - Q0 > a.qcap;
    if (tid == 0) a.tile_bad[t] = skip;
    if (skip) continue;
    const uintptr_t d0 = oq_abs + (qa - Q0), d1 = oq_abs + (qb - Q0);
    for (uintptr_t c = (d0 & ~(uintptr_t)15) + 16ull * tid; c < d1; c += 16ull * 256) {
      const uint64_t x = qa + (c - d0);  // input offset of byte c (c may precede d0)
      if (c >= d0 && c + 16 <= d1) {
        *(uint4*)c = ld16_any(a.qual, x);
      } else {
        for (int j = 0; j < 16; j++)
          if (c + j >= d0 && c + j < d1) *(uint8_t*)(c + j) = a.qual[x + j];
      }
    }
  }
}

// Values, after k_compact_classify: row r's output (region [s, e) = its input
// value bytes + 1, placed at row_val_off[r] - V0 + r) is its input with the
// 4-byte zero prefix of each legacy float removed (the row's holes: output
// positions h, in(y) = row_val_off[r] + y + 4 * #{h <= y}), then its meta
// byte 0; the 4 * holes bytes after the meta byte are unused. One row per
// 16-lane quarter wave; every aligned 16-B output chunk is written once, by
// the row holding its first byte (with the next row's head when the row ends
// inside it). Chunks crossing two row ends or two holes go byte by byte.
// Rows with offsets out of bounds write nothing (the row kernel fails the
// call on them).
struct CvRow {
  uint64_t s, e, in;  // output region [s, e), input offset of the first byte
  uint32_t h0, h1;
  bool ok;
};
DEVI CvRow cv_row(const CompactArgs& a, uint64_t r, uint64_t V0) {
  CvRow w;
  const uint64_t v0 = a.row_val_off[r], v1 = a.row_val_off[r + 1];
  const uint2 h = a.row_holes[r];
  w.ok = v0 >= V0 && v1 >= v0 && v1 <= a.val_nbytes && v1 - V0 + r + 1 <= a.vcap;
  w.s = v0 - V0 + r;
  w.e = v1 - V0 + r + 1;
  w.in = v0;
  w.h0 = h.x;
  w.h1 = h.y;
  return w;
}
DEVI uint64_t cv_meta(const CvRow& w) { return w.e - 1 - 4ull * ((w.h0 != ~0u) + (w.h1 != ~0u)); }

// One aligned 16-B output chunk c (absolute address) whose first byte lies in
// row r (w; n = row r + 1, when there is one): one source, one hole or the
// row end inside (two sources selected by byte), or byte by byte.
struct CvGlobal {
  const uint8_t* v;
  DEVI uint4 v16(uint64_t x) const { return ld16_any(v, x); }
  DEVI uint8_t b(uint64_t x) const { return v[x]; }
};
// (row_at(ru, u): row ru's CvRow into u, false past the rows the caller may
// write: the batch's, or a piece's in k_compact_plain)
// (src.v16(x) / src.b(x): 16 bytes / the byte at input value offset x, from
// global memory or a block's LDS copy)
template <class RowAt, class Src>
DEVI void cv_chunk_t(const CompactArgs& a, uint64_t r, const CvRow& w, const CvRow& n, uintptr_t c,
                     uintptr_t ov_abs, bool act, RowAt row_at, const Src& src) {
  const uint64_t m = cv_meta(w);
  const uint64_t o = c - ov_abs, y0 = o - w.s, x = w.in + y0;
  const uint64_t xa = x + 4 * ((w.h0 <= y0) + (w.h1 <= y0));
  const bool in0 = w.h0 > y0 && w.h0 < y0 + 16, in1 = w.h1 > y0 && w.h1 < y0 + 16;  // holes inside
  // one source, or one hole inside (from it on, 4 bytes further down the input)
  const bool c1 = o + 16 <= m && !(in0 && in1);
  // the meta byte at m - o; then the unused bytes; then the next row (one
  // byte further down the input; 4 more when its first KV is a legacy
  // float), which must have no hole and no end inside the chunk
  uint64_t xb = x - 1;
  bool ok = true;
  if (w.e < o + 16) {
    const uint64_t L = o + 16 - w.e;
    ok = r + 1 < a.n_rows && n.ok && !(n.h0 > 0 && n.h0 < L) && !(n.h1 > 0 && n.h1 < L) && cv_meta(n) >= o + 16;
    if (n.h0 == 0) xb += 4;
  }
  const bool c2 = !c1 && m < o + 16 && !in0 && !in1 && ok && xb + 1 != 0;  // (B inside the buffer)
  if (act && (c1 || c2)) {
    const uint64_t xB = c1 ? xa + 4 : xb;
    const int pos = c1 ? (in0 ? (int)(w.h0 - y0) : in1 ? (int)(w.h1 - y0) : 16) : (int)(m - o);
    *(uint4*)c = cq_funnel(src.v16(xa), src.v16(xB), pos, !c1);
  } else if (act) {  // byte by byte, walking the rows (two boundaries in the chunk)
    CvRow u = w;
    uint64_t ru = r;
    for (int b = 0; b < 16; b++) {
      const uint64_t ob = o + b;
      while (ob >= u.e && u.ok)
        if (!row_at(++ru, u)) u.ok = false;
      if (!u.ok) break;
      const uint64_t mu = cv_meta(u);
      if (ob > mu) continue;  // (unused)
      const uint64_t y = ob - u.s;
      *(uint8_t*)(c + b) = ob == mu ? (uint8_t)0 : src.b(u.in + y + 4 * ((u.h0 <= y) + (u.h1 <= y)));
    }
  }
}

DEVI void cv_chunk(const CompactArgs& a, uint64_t r, const CvRow& w, const CvRow& n, uintptr_t c,
                   uintptr_t ov_abs, uint64_t V0, bool act) {
  cv_chunk_t(
      a, r, w, n, c, ov_abs, act,
      [&](uint64_t ru, CvRow& u) {
        if (ru >= a.n_rows) return false;
        u = cv_row(a, ru, V0);
        return true;
      },
      CvGlobal{a.val});
}

__global__ void __launch_bounds__(256) k_compact_vals(CompactArgs a) {
  const int lane = lane_id(), sub = lane & 15, qtr = lane >> 4;
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  const uint64_t V0 = a.row_val_off[0];
  const uint64_t n_quads = (a.n_rows + 3) / 4;
  const uintptr_t ov_abs = (uintptr_t)a.ov;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + threadIdx.x / WAVE; g < n_quads; g += nw) {
    const uint64_t r = 4 * g + qtr;
    CvRow w = {}, n = {};
    uint64_t nch = 0;
    uintptr_t c0 = 0;
    if (r < a.n_rows) {
      w = cv_row(a, r, V0);
      if (r + 1 < a.n_rows) n = cv_row(a, r + 1, V0);
      if (w.ok) {  // chunks whose first byte is in [s, e)
        c0 = (ov_abs + w.s + 15) & ~(uintptr_t)15;
        nch = ov_abs + w.e > c0 ? (ov_abs + w.e - c0 + 15) / 16 : 0;
      }
    }
    const uint64_t m = cv_meta(w);
    // (branch-light: the scalar unit, shared by the CU's waves, bounded the
    // branchy version — 780 SALU per wave)
    for (uint64_t i0 = 0; ballot(i0 < nch); i0 += 16) {
      const uint64_t k = i0 + sub;
      const bool act = k < nch;
      const uintptr_t c = c0 + 16 * k;
      cv_chunk(a, r, w, n, c, ov_abs, V0, act);
    }
  }
}

// The same copy, flat: a block per run of CV_ROWS rows writes the aligned
// 16-B chunks whose first byte lies in those rows (their output is one
// contiguous range), a thread per chunk, its row found by a binary search
// over the rows' output starts in LDS — instead of a quarter wave per row
// looping over its ~19 chunks (two rounds, the second mostly idle lanes).
// A run holding a row with offsets out of bounds goes row by row.
#ifndef CV_ROWS
#define CV_ROWS 64
#endif
__global__ void __launch_bounds__(256) k_compact_vals_flat(CompactArgs a) {
  __shared__ CvRow s_w[CV_ROWS + 1];
  __shared__ uint32_t s_bad;
  const uint64_t V0 = a.row_val_off[0];
  const uintptr_t ov_abs = (uintptr_t)a.ov;
  const uint64_t nrun = (a.n_rows + CV_ROWS - 1) / CV_ROWS;
  const uint32_t t = threadIdx.x;
  for (uint64_t run = blockIdx.x; run < nrun; run += gridDim.x) {
    const uint64_t r0 = run * CV_ROWS;
    const uint32_t nr = (uint32_t)min((uint64_t)CV_ROWS, a.n_rows - r0);
    __syncthreads();  // (the previous run's rows consumed)
    if (t == 0) s_bad = 0;
    __syncthreads();
    if (t <= nr && r0 + t < a.n_rows) {  // the run's rows and the one after it
      const CvRow w = cv_row(a, r0 + t, V0);
      s_w[t] = w;
      if (t < nr && !w.ok) s_bad = 1;
    }
    __syncthreads();
    if (s_bad) {  // row by row: a wave a row, a lane a chunk
      for (uint32_t i = t / WAVE; i < nr; i += 256 / WAVE) {
        const CvRow w = s_w[i];
        if (!w.ok) continue;
        CvRow n = {};
        if (r0 + i + 1 < a.n_rows) n = s_w[i + 1];
        const uintptr_t c0 = (ov_abs + w.s + 15) & ~(uintptr_t)15;
        const uint64_t nch = ov_abs + w.e > c0 ? (ov_abs + w.e - c0 + 15) / 16 : 0;
        for (uint64_t k = lane_id(); k < nch; k += WAVE) cv_chunk(a, r0 + i, w, n, c0 + 16 * k, ov_abs, V0, true);
      }
      continue;
    }
    // every row of the run in bounds: consecutive rows' output ranges abut
    const uintptr_t cb = (ov_abs + s_w[0].s + 15) & ~(uintptr_t)15;
    const uintptr_t ce = ov_abs + s_w[nr - 1].e;
    for (uintptr_t c = cb + 16ull * t; c < ce; c += 16ull * 256) {
      const uint64_t o = c - ov_abs;
      uint32_t lo = 0, hi = nr - 1;  // the last row whose output starts at or before o
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (s_w[mid].s <= o) lo = mid; else hi = mid - 1;
      }
      CvRow n = {};
      if (r0 + lo + 1 < a.n_rows) n = s_w[lo + 1];
      cv_chunk(a, r0 + lo, s_w[lo], n, c, ov_abs, V0, true);
    }
  }
}

// ===========================================================================
// k_compact_plain: the plain-row path in one launch (round 5; the three
// kernels above stay as the "split" option). A block takes a run of CP_ROWS
// rows, in pieces whose KV lengths and row bytes fit its LDS (normally
// the whole run):
//   1. the piece's KV lengths, qualifier and value bytes staged with 16-B
//      loads (one round trip);
//   2. the plain test flat over the piece's KVs, a thread per <= 8
//      consecutive KVs: value offsets and legacy-float counts inside each row
//      from one block scan (the prefix at each row's first KV rebuilt from the
//      owning thread's exclusive prefix), the delta order, the value lengths,
//      the legacy floats' zero prefixes; the flag fix-ups patched in LDS;
//   3. per row: status / lengths / write decision (plain) or CQ_PENDING;
//   4. the qualifiers written from LDS and the values copied around the holes
//      (cv_chunk), 16-B stores; byte stores only at the piece's two edges, so
//      no two blocks write one byte.
// Every row byte is read from HBM once (the KV lengths, the qualifiers, the
// values), and the output is built from LDS. A run holding
// a row with offsets out of bounds, and a row whose bytes alone overflow the
// LDS budget, are left CQ_PENDING for k_compact_rows.
// ===========================================================================
#ifndef CP_ROWS
#define CP_ROWS 32u    // rows per run (a block iteration)
#endif
#ifndef CP_KCAP
#define CP_KCAP 2048u  // KVs per piece
#endif
#ifndef CP_QCAP
#define CP_QCAP 6144u  // qualifier bytes per piece
#endif
#ifndef CP_GRID
#define CP_GRID 65536u  // blocks (each loops over runs, the next run's offsets in flight)
#endif
#ifndef CP_THREADS
#define CP_THREADS 256u  // threads a block
#endif
constexpr uint32_t CP_KPT = CP_KCAP / CP_THREADS;  // KVs a thread
static_assert(CP_KPT == 4 || CP_KPT == 8, "k_compact_plain: 4 or 8 KVs a thread");
#ifndef CP_VCAP
#define CP_VCAP 12288u  // value bytes per piece
#endif

// the staged piece: four segments back to back in 16-B chunk order (the KV
// qualifier lengths, the KV value lengths, the qualifier bytes, the value
// bytes; each from its source's aligned 16-B chunk holding the piece's first
// byte), so that chunk c lands at buf + 16 c and one global_load_lds of a wave
// writes 64 consecutive chunks
constexpr uint32_t CP_CHUNKS = 2 * ((14 + 2 * CP_KCAP + 15) / 16) + (15 + CP_QCAP + 15) / 16 + (15 + CP_VCAP + 15) / 16;
struct __attribute__((aligned(16))) CpLds {
  uint8_t pad0[16];  // (cv_chunk's second source may start one byte before the piece's values)
  uint8_t buf[16 * CP_CHUNKS + 64];
  uint64_t kv[CP_ROWS + 1], qo[CP_ROWS + 1], vo[CP_ROWS + 1];  // the run's row offsets
  CvRow w[CP_ROWS];
  // the piece's rows (index i = row - j0): first KV (relative) | plain
  // candidate (>= 2 KVs, 2 qualifier bytes each) << 31, LDS index of the
  // first qualifier byte, value bytes, first value byte (relative)
  uint4 rec[CP_ROWS];
  uint32_t pstart[CP_ROWS], pend[CP_ROWS];  // scan prefix (value bytes | legacy floats << 16) around the row's KVs
  uint32_t bad[CP_ROWS], h0[CP_ROWS], h1[CP_ROWS];
  uint8_t krow[CP_KCAP + 16];  // each KV's row
  uint32_t scan[CP_THREADS / 64];
  uint32_t insane;
};
static_assert(sizeof(CpLds) <= 80 * 1024, "k_compact_plain: 2 blocks a CU");
static_assert(CP_QCAP % 16 == 0 && CP_KCAP % 8 == 0, "16-B aligned LDS buffers");


// 16 bytes from LDS at any byte index (dword loads + alignbyte).
DEVI uint4 lds_ld16_any(const uint8_t* L, uint32_t i) {
  const uint32_t* d = (const uint32_t*)(L + (i & ~3u));
  const uint32_t sb = i & 3u;
  uint32_t v[5];
#pragma unroll
  for (int k = 0; k < 5; k++) v[k] = d[k];
  return make_uint4(__builtin_amdgcn_alignbyte(v[1], v[0], sb), __builtin_amdgcn_alignbyte(v[2], v[1], sb),
                    __builtin_amdgcn_alignbyte(v[3], v[2], sb), __builtin_amdgcn_alignbyte(v[4], v[3], sb));
}

struct CpBufs {  // the piece's segments in CpLds::buf
  const uint16_t* ql;
  const uint16_t* vl;
  uint8_t* q;  // (index: qualifier offset - the piece's first + hq)
  const uint8_t* x;  // (index: value offset - the piece's first)
};

struct CvLds {  // cv_chunk's source: the piece's value bytes in LDS
  const uint8_t* v;
  uint64_t base;  // input offset of LDS byte 0
  DEVI uint4 v16(uint64_t x) const { return lds_ld16_any(v, (uint32_t)(x - base)); }
  DEVI uint8_t b(uint64_t x) const { return v[x - base]; }
};

// The block barrier of k_compact_plain. (A barrier waiting for LDS only —
// s_waitcnt lgkmcnt(0) + s_barrier, not for the global stores before it —
// measured 1 % slower on C5 than __syncthreads, profiles/r05/c5/.)
DEVI void cp_sync() { __syncthreads(); }

// Block exclusive scan of x over cp_sync; *total the sum.
DEVI uint32_t cp_scan(uint32_t x, uint32_t& total, uint32_t* sh /* [CP_THREADS / WAVE] */) {
  const int lane = lane_id(), w = threadIdx.x / WAVE;
  const uint32_t ix = wave_incl_scan_u32_dpp(x);
  if (lane == 63) sh[w] = ix;
  cp_sync();
  uint32_t p = 0;
  total = 0;
#pragma unroll
  for (int k = 0; k < (int)(CP_THREADS / WAVE); k++) {
    if (k < w) p += sh[k];
    total += sh[k];
  }
  return p + ix - x;
}

// One piece [j0, j1) of the run starting at row r0.
DEVI void cp_piece(const CompactArgs& a, CpLds& L, uint64_t r0, uint32_t j0, uint32_t j1, uint64_t Q0, uint64_t V0) {
  const uint32_t t = threadIdx.x, np = j1 - j0;
  const uint64_t KA = L.kv[j0], QA = L.qo[j0], QB = L.qo[j1], VA = L.vo[j0], VB = L.vo[j1];
  const uint32_t NK = (uint32_t)(L.kv[j1] - KA);
  cp_sync();  // (the previous piece's LDS consumed)
  // ---- 1. staging: KV lengths, qualifier bytes (16-B loads, several in flight) ----
  const uintptr_t sk = (uintptr_t)(a.kv_qual_len + KA), sv = (uintptr_t)(a.kv_val_len + KA), sq = (uintptr_t)(a.qual + QA);
  const uintptr_t sx = (uintptr_t)(a.val + VA);
  const uint32_t hkb = (uint32_t)(sk & 15u), hvb = (uint32_t)(sv & 15u), hq = (uint32_t)(sq & 15u);
  const uint32_t hx = (uint32_t)(sx & 15u);
  const uint32_t nk1 = NK ? (hkb + 2 * NK + 15) / 16 : 0u, nv1 = NK ? (hvb + 2 * NK + 15) / 16 : 0u;
  const uint32_t nq1 = QB > QA ? (uint32_t)((hq + (QB - QA) + 15) / 16) : 0u;
  const uint32_t nx1 = VB > VA ? (uint32_t)((hx + (VB - VA) + 15) / 16) : 0u;
  const uint32_t e1 = nk1 + nv1, e2 = e1 + nq1, tot = e2 + nx1;
  // (four loads in flight a thread, then their LDS writes; global_load_lds
  // staging measured slower: profiles/r05/c5/)
  auto src = [&](uint32_t c) {
    return c < nk1  ? (const uint4*)(sk - hkb) + c
           : c < e1 ? (const uint4*)(sv - hvb) + (c - nk1)
           : c < e2 ? (const uint4*)(sq - hq) + (c - e1)
                    : (const uint4*)(sx - hx) + (c - e2);
  };
  uint4* const dst = (uint4*)L.buf;
  constexpr uint32_t T = CP_THREADS;
  for (uint32_t c = t; c < tot; c += 4 * T) {  // (four named register sets: an array lands in scratch)
    const bool b1 = c + T < tot, b2 = c + 2 * T < tot, b3 = c + 3 * T < tot;
    const uint4 v0 = *src(c);
    uint4 v1 = {}, v2 = {}, v3 = {};
    if (b1) v1 = *src(c + T);
    if (b2) v2 = *src(c + 2 * T);
    if (b3) v3 = *src(c + 3 * T);
    dst[c] = v0;
    if (b1) dst[c + T] = v1;
    if (b2) dst[c + 2 * T] = v2;
    if (b3) dst[c + 3 * T] = v3;
  }
  const CpBufs B{(const uint16_t*)(L.buf + hkb), (const uint16_t*)(L.buf + 16 * nk1 + hvb), L.buf + 16 * e1,
                 L.buf + 16 * e2 + hx};
  if (t < np) {  // the piece's rows: record, scan prefixes, flags; each KV's row index in krow
    const uint32_t j = j0 + t;
    const uint64_t nk = L.kv[j + 1] - L.kv[j];
    const uint32_t k0 = (uint32_t)(L.kv[j] - KA), k1 = (uint32_t)(L.kv[j + 1] - KA);
    const bool cand = nk >= 2 && L.qo[j + 1] - L.qo[j] == 2 * nk;
    L.rec[t] = make_uint4(k0 | (cand ? 1u << 31 : 0u), (uint32_t)(L.qo[j] - QA) + hq, (uint32_t)(L.vo[j + 1] - L.vo[j]),
                          (uint32_t)(L.vo[j] - VA));
    L.pstart[t] = L.pend[t] = 0;
    L.bad[t] = 0;
    L.h0[t] = L.h1[t] = ~0u;
    uint32_t k = k0;
    for (; k < k1 && (k & 3u); k++) L.krow[k] = (uint8_t)t;
    for (; k + 4 <= k1; k += 4) *(uint32_t*)(L.krow + k) = t * 0x01010101u;
    for (; k < k1; k++) L.krow[k] = (uint8_t)t;
  }
  cp_sync();
#ifndef CP_ABL
#define CP_ABL 0  // (ablation builds only: 1 no value copy, 2 no qualifier copy, 4 no plain test)
#endif
  // ---- 2. the plain test, flat over the KVs: a thread per 8 consecutive
  // KVs, every LDS load of the 8 issued together (no dependent walk) ----
  const uint32_t kb = CP_KPT * t;
  const bool any = kb < NK && !(CP_ABL & 4);
  uint32_t ir[CP_KPT], q_[CP_KPT], ql_[CP_KPT], vl_[CP_KPT], c_[CP_KPT], pre_[CP_KPT];
  uint32_t sum = 0;
  {
    uint32_t kr[CP_KPT / 4] = {};
    uint4 ql4[(CP_KPT + 7) / 8] = {}, vl4[(CP_KPT + 7) / 8] = {};
    if (any) {
#pragma unroll
      for (int w = 0; w < (int)(CP_KPT / 4); w++) kr[w] = *(const uint32_t*)(L.krow + kb + 4 * w);
#pragma unroll
      for (int w = 0; w < (int)((CP_KPT + 7) / 8); w++) {
        ql4[w] = lds_ld16_any((const uint8_t*)B.ql, 2 * kb + 16 * w);
        vl4[w] = lds_ld16_any((const uint8_t*)B.vl, 2 * kb + 16 * w);
      }
    }
#pragma unroll
    for (int u = 0; u < (int)CP_KPT; u++) {
      const uint32_t k = kb + u;
      const bool act = k < NK;
      const uint32_t qw = u % 8 < 2 ? ql4[u / 8].x : u % 8 < 4 ? ql4[u / 8].y : u % 8 < 6 ? ql4[u / 8].z : ql4[u / 8].w;
      const uint32_t vw = u % 8 < 2 ? vl4[u / 8].x : u % 8 < 4 ? vl4[u / 8].y : u % 8 < 6 ? vl4[u / 8].z : vl4[u / 8].w;
      ir[u] = (kr[u / 4] >> (8 * (u % 4))) & 0xFFu;
      ql_[u] = act ? (qw >> (16 * (u % 2))) & 0xFFFFu : 0u;
      vl_[u] = act ? (vw >> (16 * (u % 2))) & 0xFFFFu : 0u;
      q_[u] = 0;
      c_[u] = 0;
      if (act) {
        const uint4 R = L.rec[ir[u]];
        if ((R.x >> 31) && ql_[u] == 2) q_[u] = lds_q16(B.q, R.y + 2 * (k - (R.x & 0x7FFFFFFFu)));
        const bool leg = (R.x >> 31) && ql_[u] == 2 && cq_legacy(q_[u] & 0xFFu, vl_[u]);  // :510-515
        c_[u] = min(vl_[u], 9u) | (leg ? 1u << 16 : 0u);
      }
      pre_[u] = sum;  // (exclusive, inside the thread)
      sum += c_[u];
    }
  }
  uint32_t tx;
  const uint32_t ex = cp_scan(sum, tx, L.scan);
  // each row's scan prefix before its first KV and after its last, by the
  // threads owning those KVs (a row without KVs is not plain: never read)
  if (any) {
    const uint32_t nxt = kb + CP_KPT < NK ? L.krow[kb + CP_KPT] : 0xFFu;
#pragma unroll
    for (int u = 0; u < (int)CP_KPT; u++) {
      const uint32_t k = kb + u;
      if (k < NK) {
        const uint32_t i = ir[u];
        if (u == 0 ? (k == 0 || L.krow[k - 1] != i) : ir[u - 1] != i) L.pstart[i] = ex + pre_[u];
        if (u + 1 < (int)CP_KPT ? (k + 1 >= NK || ir[u + 1] != i) : (k + 1 >= NK || nxt != i))
          L.pend[i] = ex + pre_[u] + c_[u];
      }
    }
  }
  cp_sync();
  if (any) {
#pragma unroll
    for (int u = 0; u < (int)CP_KPT; u++) {
      const uint32_t k = kb + u;
      if (k >= NK) continue;
      const uint32_t i = ir[u];
      const uint4 R = L.rec[i];
      if (!(R.x >> 31)) continue;
      const uint32_t kv_i = R.x & 0x7FFFFFFFu;
      const uint32_t rel = ex + pre_[u] - L.pstart[i], vin = rel & 0xFFFFu, nl = rel >> 16;
      const uint32_t ql = ql_[u], vl = vl_[u], q = q_[u];
      const bool leg = (c_[u] >> 16) != 0;
      const uint32_t qpos = R.y + 2 * (k - kv_i);
      bool kbad = ql != 2 || vl == 0 || vl > 8;
      if (!kbad && k > kv_i) {  // deltas strictly increasing (the KV before is in the row)
        const uint32_t qp = u > 0 ? q_[u > 0 ? u - 1 : 0] : lds_q16(B.q, qpos - 2);
        kbad = (q >> 4) <= (qp >> 4);
      }
      if (!kbad) kbad = vin + vl > R.z;
      if (leg && !kbad) {  // the 4-byte zero prefix (fixFloatingPointValue :530-544)
        const uint8_t* vp = B.x + R.w + vin;
        kbad = (vp[0] | vp[1] | vp[2] | vp[3]) != 0;
      }
      if (!kbad) {  // fixQualifierFlags :490-499 (delta bits unchanged: a neighbour's order check
                    // reads the same delta before or after the patch)
        const uint8_t f = (uint8_t)cq_fixq(q & 0xFFu, leg ? 4u : vl);
        if (f != (uint8_t)q) B.q[qpos + 1] = f;
      } else {
        L.bad[i] = 1;
      }
      if (leg) {  // the holes: output positions of the row's first two legacy floats
        if (nl == 0) L.h0[i] = vin;
        else if (nl == 1) L.h1[i] = vin - 4;
      }
    }
  }
  cp_sync();
  // ---- 3. the rows' results ----
  if (t < np) {
    const uint32_t j = j0 + t;
    const uint64_t r = r0 + j;
    const uint4 R = L.rec[t];
    const uint32_t d = L.pend[t] - L.pstart[t], vsum = d & 0xFFFFu, legs = d >> 16;
    const bool plain = (R.x >> 31) && !L.bad[t] && legs <= 2 && vsum == R.z;
    CvRow w;
    w.s = L.vo[j] - V0 + r;
    w.e = L.vo[j + 1] - V0 + r + 1;
    w.in = L.vo[j];
    w.h0 = plain ? L.h0[t] : ~0u;
    w.h1 = plain ? L.h1[t] : ~0u;
    w.ok = true;
    L.w[t] = w;
    if (plain) {
      a.out_qoff[r] = L.qo[j] - Q0;
      a.out_voff[r] = w.s;
      cq_finish(a, r, CQ_TRIVIAL, (uint32_t)(L.qo[j + 1] - L.qo[j]), vsum - 4 * legs + 1);
    } else {
      a.status[r] = CQ_PENDING;  // (to the LDS row kernel)
    }
  }
  cp_sync();
  // ---- 4. qualifiers from LDS, values around the holes ----
  {
    const uintptr_t d0 = (uintptr_t)a.oq + (QA - Q0), d1 = (uintptr_t)a.oq + (QB - Q0);
    const uintptr_t c0 = (d0 + 15) & ~(uintptr_t)15, c1 = d1 & ~(uintptr_t)15;
    for (uintptr_t c = c0 + 16ull * t; c < c1 && !(CP_ABL & 2); c += 16ull * CP_THREADS)
      *(uint4*)c = lds_ld16_any(B.q, (uint32_t)(c - d0) + hq);
    const uintptr_t he = c0 < d1 ? c0 : d1, ts = c1 > he ? c1 : he;  // edge bytes [d0, he), [ts, d1)
    const uintptr_t x = t < 16 ? d0 + t : ts + (t - 16);
    if ((t < 16 && x < he) || (t >= 16 && t < 32 && x < d1)) *(uint8_t*)x = B.q[(uint32_t)(x - d0) + hq];
  }
  {
    const uintptr_t ov_abs = (uintptr_t)a.ov;
    const uintptr_t d0 = ov_abs + L.w[0].s, d1 = ov_abs + L.w[np - 1].e;
    const uintptr_t c0 = (d0 + 15) & ~(uintptr_t)15, c1 = d1 & ~(uintptr_t)15;
    auto row_at = [&](uint64_t ru, CvRow& u) {
      if (ru >= r0 + j1) return false;
      u = L.w[ru - r0 - j0];
      return true;
    };
    auto find = [&](uint64_t o) {  // the piece's last row whose output starts at or before o
      uint32_t lo = 0, hi = np - 1;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (L.w[mid].s <= o) lo = mid; else hi = mid - 1;
      }
      return lo;
    };
    const CvLds xs{L.pad0, VA - 16 - 16 * e2 - hx};
    for (uintptr_t c = c0 + 16ull * t; c < c1 && !(CP_ABL & 1); c += 16ull * CP_THREADS) {
      const uint32_t i = find(c - ov_abs);
      CvRow n = {};
      if (i + 1 < np) n = L.w[i + 1];
      cv_chunk_t(a, r0 + j0 + i, L.w[i], n, c, ov_abs, true, row_at, xs);
    }
    const uintptr_t he = c0 < d1 ? c0 : d1, ts = c1 > he ? c1 : he;
    const uintptr_t x = t < 16 ? d0 + t : ts + (t - 16);
    if ((t < 16 && x < he) || (t >= 16 && t < 32 && x < d1)) {
      const uint64_t o = x - ov_abs;
      const CvRow& u = L.w[find(o)];
      const uint64_t m = cv_meta(u), y = o - u.s;
      if (o <= m) *(uint8_t*)x = o == m ? (uint8_t)0 : xs.b(u.in + y + 4 * ((u.h0 <= y) + (u.h1 <= y)));
    }
  }
}

__global__ void __launch_bounds__(CP_THREADS) k_compact_plain(CompactArgs a) {
  __shared__ CpLds L;
  const uint32_t t = threadIdx.x;
  const uint64_t Q0 = a.row_qual_off[0], V0 = a.row_val_off[0];
  const uint64_t nrun = (a.n_rows + CP_ROWS - 1) / CP_ROWS;
  // the next run's row offsets are loaded while this run is compacted
  uint64_t hk = 0, hq = 0, hv = 0;
  auto fetch = [&](uint64_t rn) {
    if (rn < nrun && t <= min((uint64_t)CP_ROWS, a.n_rows - rn * CP_ROWS)) {
      hk = a.row_kv_start[rn * CP_ROWS + t];
      hq = a.row_qual_off[rn * CP_ROWS + t];
      hv = a.row_val_off[rn * CP_ROWS + t];
    }
  };
  fetch(blockIdx.x);
  for (uint64_t run = blockIdx.x; run < nrun; run += gridDim.x) {
    const uint64_t r0 = run * CP_ROWS;
    const uint32_t nr = (uint32_t)min((uint64_t)CP_ROWS, a.n_rows - r0);
    cp_sync();  // (the previous run's LDS consumed)
    if (t <= nr) {
      L.kv[t] = hk;
      L.qo[t] = hq;
      L.vo[t] = hv;
    }
    fetch(run + gridDim.x);
    if (t == 0) L.insane = 0;
    cp_sync();
    if (t < nr) {  // the row's offsets in bounds (then its ranges are disjoint from every other row's)
      const uint64_t r = r0 + t;
      const uint64_t kv = L.kv[t], kv_n = L.kv[t + 1], qo = L.qo[t], qo_n = L.qo[t + 1], vo = L.vo[t], vo_n = L.vo[t + 1];
      const bool sane = kv_n >= kv && kv_n <= a.n_kvs && qo_n >= qo && vo_n >= vo && qo >= Q0 && vo >= V0 &&
                        qo_n <= a.qual_nbytes && vo_n <= a.val_nbytes && qo_n - Q0 <= a.qcap &&
                        vo_n - V0 + r + 1 <= a.vcap && vo_n - vo < (1ull << 32);
      if (!sane) L.insane = 1;
    }
    cp_sync();
    if (L.insane) {  // the whole run to the row kernel (which finds the bad offsets)
      if (t < nr) a.status[r0 + t] = CQ_PENDING;
      continue;
    }
    uint32_t j0 = 0;
    while (j0 < nr) {  // (uniform)
      uint32_t lo = j0, hi = nr;  // the most rows from j0 whose KVs and qualifier bytes fit
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) >> 1;
        if (L.kv[mid] - L.kv[j0] <= CP_KCAP && L.qo[mid] - L.qo[j0] <= CP_QCAP && L.vo[mid] - L.vo[j0] <= CP_VCAP)
          lo = mid;
        else
          hi = mid - 1;
      }
      if (lo == j0) {  // one row over the budget alone
        if (t == 0) a.status[r0 + j0] = CQ_PENDING;
        j0++;
        continue;
      }
      cp_piece(a, L, r0, j0, lo, Q0, V0);
      j0 = lo;
    }
  }
}

// The listed (non-plain) rows through cq_row_lds, CT_ROWS per block at a
// time, each row staged into its own LDS ranges (16-B loads) and written back
// from its own output ranges (16-B stores inside the row); rows over the LDS
// budget go through cq_row_global.
DEVI void cq_unstage_wave(uint8_t* dst, const uint8_t* lds, uint32_t i0, uint64_t b0, uint64_t b1, int lane) {
  if (b1 <= b0) return;
  const uintptr_t s = (uintptr_t)(dst + b0), e = (uintptr_t)(dst + b1);
  const uintptr_t a0 = (s + 15) & ~(uintptr_t)15, a1 = e & ~(uintptr_t)15;  // whole chunks [a0, a1)
  if (a0 < a1) {
    for (uintptr_t cs = a0 + 16ull * lane; cs < a1; cs += 16ull * WAVE)
      *(uint4*)cs = *(const uint4*)(lds + i0 + (cs - s));
  }
  // the partial chunks at either end, one byte per lane (lanes 0-15 head,
  // 16-31 tail; one range when the row lies inside a single chunk)
  const uintptr_t h1 = a0 < e ? a0 : e;
  const uintptr_t t0 = a1 > h1 ? a1 : h1;
  uintptr_t x = 0;
  if (lane < 16) x = s + lane;
  else if (lane < 32) x = t0 + (lane - 16);
  if ((lane < 16 && x < h1) || (lane >= 16 && lane < 32 && x < e)) dst[x - (uintptr_t)dst] = lds[i0 + (x - s)];
}
DEVI uint32_t cq_need(uint64_t len) { return (uint32_t)((len + 15 + 15) & ~15ull); }  // staged: head <= 15

#ifndef CR_RANGE
#define CR_RANGE 256u  // rows scanned for CQ_PENDING per block iteration
#endif

__global__ void __launch_bounds__(256) k_compact_rows(CompactArgs a) {
  __shared__ TileLds L;
  __shared__ RowHdr s_h[CT_ROWS];
  __shared__ RowLds s_p[CT_ROWS];
  __shared__ uint32_t s_fit[CT_ROWS];
  // staging segments, l = 4 * row + stream (qualifiers, values, qualifier
  // lengths, value lengths): aligned source, LDS byte offset, first chunk
  __shared__ const uint4* s_src[4 * CT_ROWS];
  __shared__ uint32_t s_dst[4 * CT_ROWS], s_c0[4 * CT_ROWS + 1];
  __shared__ uint32_t s_list[CR_RANGE], s_wn[4];
  static_assert(4 * CT_ROWS == WAVE, "one staging segment per lane of wave 0");
  const int tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
  const uint64_t Q0 = a.row_qual_off[0], V0 = a.row_val_off[0];
  uint8_t* const Lb = (uint8_t*)&L;
  if (tid == 0) L.n_complex = 0;
  for (uint64_t rb = (uint64_t)blockIdx.x * CR_RANGE; rb < a.n_rows; rb += (uint64_t)gridDim.x * CR_RANGE) {
    // ---- the range's CQ_PENDING rows, in row order, into s_list ----
    __syncthreads();  // (the previous range's list consumed)
    constexpr int CR_U = CR_RANGE >= 256 ? (int)(CR_RANGE / 256) : 1;  // (ranges of 64 / 128 rows: lanes idle)
    uint32_t pend[CR_U], wpos = 0;
#pragma unroll
    for (int u = 0; u < CR_U; u++) {
      const uint32_t q = u * WAVE + lane;  // (wave w: a quarter of the range)
      const uint64_t r = rb + (uint64_t)w * (CR_RANGE / 4) + q;
      const bool pd = q < CR_RANGE / 4 && r < a.n_rows && a.status[r] == CQ_PENDING;
      const uint64_t m = ballot(pd);
      pend[u] = pd ? wpos + (uint32_t)__popcll(m & lanemask_lt(lane)) : ~0u;
      wpos += (uint32_t)__popcll(m);
    }
    if (lane == 0) s_wn[w] = wpos;
    __syncthreads();
    uint32_t woff = 0;
    for (int v = 0; v < w; v++) woff += s_wn[v];
    const uint32_t n = s_wn[0] + s_wn[1] + s_wn[2] + s_wn[3];
#pragma unroll
    for (int u = 0; u < CR_U; u++)
      if (pend[u] != ~0u) s_list[woff + pend[u]] = (uint32_t)(rb + (uint64_t)w * (CR_RANGE / 4) + u * WAVE + lane);
    const uint32_t* list = s_list;
  for (uint32_t t = 0; t * CT_ROWS < n; t++) {
    const uint32_t nr = min((uint32_t)CT_ROWS, n - t * CT_ROWS);
    __syncthreads();  // (the previous tile's LDS consumed; s_list written)
    if (w == 0) {
      // ---- LDS ranges of each row, in order, while they fit ----
      RowHdr h = {};
      uint32_t nq = 0, nv = 0, nk = 0, noq = 0, nov = 0;
      bool ok = false;
      if ((uint32_t)lane < nr) {
        h = cq_row(a, list[t * CT_ROWS + lane]);
        s_h[lane] = h;
        const uint32_t phq = (uint32_t)((uintptr_t)(a.oq + h.oqo) & 15u);
        const uint32_t phv = (uint32_t)((uintptr_t)(a.ov + h.ovo) & 15u);
        const uint64_t ql = h.qe - h.qs, vl = h.ve - h.vs;
        ok = h.ok && h.qe >= h.qs && h.ve >= h.vs && ql <= CT_QB && vl <= CT_VB && h.nk <= CT_KB;
        if (ok) {
          nq = cq_need(ql);
          nv = cq_need(vl);
          nk = cq_need(2 * h.nk);
          noq = (uint32_t)((phq + ql + 15) & ~15ull);
          nov = (uint32_t)((phv + vl + 1 + 15) & ~15ull);
        }
        h.oqo = phq;  // (kept for the output positions below)
        h.ovo = phv;
      }
      uint32_t bq = 0, bv = 0, bk = 0, boq = 0, bov = 0;  // (wave-uniform)
      RowLds p = {};
      bool fit = false;
      for (uint32_t j = 0; j < nr; j++) {
        const uint32_t jq = readlane_u32(nq, j), jv = readlane_u32(nv, j), jk = readlane_u32(nk, j);
        const uint32_t joq = readlane_u32(noq, j), jov = readlane_u32(nov, j);
        const bool f = readlane_u32(ok, j) && bq + jq <= CT_QB && bv + jv <= CT_VB && bk + jk <= 2 * CT_KB &&
                       boq + joq <= CT_QB && bov + jov <= CT_VB;
        if (lane == (int)j) {
          fit = f;
          p.k0 = p.kv0 = bk;  // (+ each source's head, once staged)
          p.qi = bq;
          p.vi = bv;
          p.qo = boq + (uint32_t)h.oqo;
          p.vo = bov + (uint32_t)h.ovo;
        }
        if (f) { bq += jq; bv += jv; bk += jk; boq += joq; bov += jov; }
      }
      if ((uint32_t)lane < nr) {
        s_fit[lane] = fit;
        s_p[lane] = p;
      }
      wave_lds_sync();
      // ---- staging segments ----
      const uint32_t j = (uint32_t)lane >> 2, sg = (uint32_t)lane & 3;
      uint32_t nch = 0, dst = 0;
      const uint8_t* src = nullptr;
      if (j < nr && s_fit[j]) {
        const RowHdr hj = s_h[j];
        const RowLds pj = s_p[j];
        uint64_t b0, b1;
        if (sg == 0) { src = a.qual; b0 = hj.qs; b1 = hj.qe; dst = (uint32_t)(L.qin - Lb) + pj.qi; }
        else if (sg == 1) { src = a.val; b0 = hj.vs; b1 = hj.ve; dst = (uint32_t)(L.vin - Lb) + pj.vi; }
        else {
          src = (const uint8_t*)(sg == 2 ? a.kv_qual_len : a.kv_val_len);
          b0 = 2 * hj.kb;
          b1 = 2 * (hj.kb + hj.nk);
          dst = (uint32_t)((sg == 2 ? L.qlen : L.vlen) - Lb) + pj.k0;
        }
        const uintptr_t sp = (uintptr_t)(src + b0);
        const uint32_t head = (uint32_t)(sp & 15u);
        nch = b1 > b0 ? (uint32_t)((head + (b1 - b0) + 15) / 16) : 0u;
        src = (const uint8_t*)(sp - head);
      }
      const uint32_t inc = wave_incl_scan_u32_dpp(nch);
      s_src[lane] = (const uint4*)src;
      s_dst[lane] = dst;
      s_c0[lane] = inc - nch;
      if (lane == WAVE - 1) s_c0[WAVE] = inc;
    }
    __syncthreads();
    // ---- stage the fitting rows: every 16-B chunk of every segment, four
    // loads in flight per thread ----
    {
      const uint32_t total = s_c0[WAVE];
      // (four named register sets: an indexed array of them lands in scratch)
      auto locate = [&](uint32_t cc, const uint4*& src, uint32_t& dst) {
        uint32_t lo = 0;  // the last segment starting at or before cc
#pragma unroll
        for (int st = 32; st > 0; st >>= 1)
          if (s_c0[lo + st] <= cc) lo += st;
        src = s_src[lo] + (cc - s_c0[lo]);
        dst = s_dst[lo] + 16 * (cc - s_c0[lo]);
      };
      for (uint32_t c = tid; c < total; c += 4 * 256) {
        const uint4 *p0 = nullptr, *p1 = nullptr, *p2 = nullptr, *p3 = nullptr;
        uint32_t d0 = 0, d1 = 0, d2 = 0, d3 = 0;
        const bool b0 = c < total, b1 = c + 256 < total, b2 = c + 512 < total, b3 = c + 768 < total;
        if (b0) locate(c, p0, d0);
        if (b1) locate(c + 256, p1, d1);
        if (b2) locate(c + 512, p2, d2);
        if (b3) locate(c + 768, p3, d3);
        uint4 v0 = {}, v1 = {}, v2 = {}, v3 = {};
        if (b0) v0 = *p0;
        if (b1) v1 = *p1;
        if (b2) v2 = *p2;
        if (b3) v3 = *p3;
        if (b0) *(uint4*)(Lb + d0) = v0;
        if (b1) *(uint4*)(Lb + d1) = v1;
        if (b2) *(uint4*)(Lb + d2) = v2;
        if (b3) *(uint4*)(Lb + d3) = v3;
      }
    }
    __syncthreads();
    // ---- compact (wave per row), unstage its own output ----
    for (uint32_t j = w; j < nr; j += 4) {
      const uint64_t r = list[t * CT_ROWS + j];
      const RowHdr h = s_h[j];
      if (lane == 0) {
        a.out_qoff[r] = h.oqo;
        a.out_voff[r] = h.ovo;
      }
      if (!s_fit[j]) {
        cq_row_global(a, r, lane);
        continue;
      }
      RowLds p = s_p[j];
      p.qi += (uint32_t)((uintptr_t)(a.qual + h.qs) & 15u);  // (cq_stage's head)
      p.vi += (uint32_t)((uintptr_t)(a.val + h.vs) & 15u);
      p.k0 += (uint32_t)((uintptr_t)((const uint8_t*)a.kv_qual_len + 2 * h.kb) & 15u);
      p.kv0 += (uint32_t)((uintptr_t)((const uint8_t*)a.kv_val_len + 2 * h.kb) & 15u);
      uint32_t oql = 0, ovl = 0;
      if (!cq_row_lds(a, r, h, L, p, L.keys[w], L.pay[w], L.runs[w], lane, &oql, &ovl)) continue;
      wave_lds_sync();
      cq_unstage_wave(a.oq, L.qout, p.qo, h.oqo, h.oqo + oql, lane);
      cq_unstage_wave(a.ov, L.vout, p.vo, h.ovo, h.ovo + ovl, lane);
    }
  }
  }
  __syncthreads();
  if (tid == 0 && L.n_complex) atomicAdd(&a.counters[3], L.n_complex);
}
}  // namespace tsdb
