// k_compact.hip — CompactionQueue.compact(row, compacted) on gfx950
// (reference: src/core/CompactionQueue.java:243-743), the secondary path.
//
// Launches over a batch of rows (tsdbhip_rows_desc), in this order:
//   k_compact_wave     the plain rows (round 6, see its comment below): one
//                      wave per run of CW_ROWS consecutive rows, staged in the
//                      wave's own LDS with 16-B loads; the plain-row test flat
//                      over the run's KVs; plain rows' results and the run's
//                      qualifier / value output written back with 16-B
//                      stores; every other row left CQ_PENDING. Wave-level LDS
//                      syncs only: no block barrier, so the CU's resident
//                      waves overlap each other's staging, tests and stores;
//   k_compact_rows     the CQ_PENDING rows, gathered per range of CR_RANGE rows,
//                      a wave per row: staged into the wave's LDS, the whole
//                      compact() of the row (single KVs, junk, errors,
//                      complexCompact of <= CW_SORT cells) and its write/delete
//                      decision from that copy; rows over its budget through
//                      cq_row_global, bigger complex rows listed for
//   k_compact_complex  one 256-thread block per complex row of more than
//                      CW_SORT cells: breakDownValues (:690-743) into a cell
//                      table (LDS, or global scratch for rows over
//                      LDS_CELLS cells), then the stable sort + duplicate
//                      check of complexCompact (:600-679) as a 4096-slot
//                      table indexed by the 12-bit time delta: slot[delta] =
//                      first cell (atomicMin); every other cell of that delta
//                      must equal it byte for byte (same q[1], same value) or
//                      the row is an IllegalDataException. Emission walks the
//                      slots in delta order, which is the sorted order;
//   k_compact_dups     the write/delete decision of the rows k_compact_complex
//                      (or cq_row_global) finished COMPLEX.
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
constexpr uint8_t CQ_PENDING = 0xFF;  // (k_compact_wave: left to k_compact_rows)

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
                        // [3] rows k_compact_rows took to complexCompact in-wave
  uint32_t* list_lds;   // complex rows with <= CQ_LDS_CELLS cells
  uint32_t* list_big;   // the others
  uint64_t* big_cells;  // scratch: row r's cells at (row_qual_off[r]-row_qual_off[0])/2 + r
  uint64_t* ext_out;    // optional: row_qual_off[0], [n_rows], row_val_off[0], [n_rows] for the host's checks
};
constexpr int CQ_REACHED_COMPLEX = 0x100;  // cq_row_lds: the row went through complexCompact

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
// k_compact_rows for rows that do not fit its LDS budget.
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
// The LDS row logic: one row classified exactly as compact() does (junk KVs,
// single KV, the in-order delta check of the trivial pre-pass :286-333,
// legacy floats) and compacted by one wave from LDS copies of its KV lengths,
// qualifier and value bytes, complex rows of <= SORT cells included
// (k_compact_rows: a wave per pending row).
// ===========================================================================
constexpr int CQ_RUNS_SLOTS = 12;

DEVI uint32_t lds_q16(const uint8_t* p, uint32_t i) { return ((uint32_t)p[i] << 8) | p[i + 1]; }
DEVI uint32_t lds_u16(const uint8_t* p, uint32_t i) { return (uint32_t)p[i] | ((uint32_t)p[i + 1] << 8); }

// A row's LDS buffers. qout may be qin itself (k_compact_wave writes a row's
// compacted qualifier over its input: every write lands at or before the
// bytes still to be read).
struct RowBufs {
  const uint8_t* qlen;  // KV qualifier lengths (u16, little-endian as staged)
  const uint8_t* vlen;  // KV value lengths
  const uint8_t* qin;
  const uint8_t* vin;
  uint8_t* qout;
  uint8_t* vout;
  uint32_t qlim, vlim;  // clamps of qin / vin indices (reads past them stay inside the LDS block)
};

// Row positions inside the buffers.
struct RowLds {
  uint32_t k0;   // byte index of the row's first KV length in qlen
  uint32_t kv0;  // ... in vlen
  uint32_t qi;   // index of the row's first qualifier byte in qin
  uint32_t vi;   // ... first value byte in vin
  uint32_t qo;   // index in qout of the row's compacted qualifier
  uint32_t vo;   // index in vout of the row's compacted value
};

// Bitonic sort (ascending) of keys[0, n) by one wave (keys has room for the
// next power of two).
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
template <uint32_t SORT>
DEVI uint8_t cq_complex_lds(const RowBufs& L, const RowLds& p, uint32_t nk, uint32_t n_single, uint32_t n_cells,
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
    uint32_t key[SORT / WAVE], rank[SORT / WAVE];
#pragma unroll
    for (int k = 0; k < (int)(SORT / WAVE); k++) {
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
    for (int k = 0; k < (int)(SORT / WAVE); k++)
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

// One row, LDS -> LDS (same classification as cq_row_global); lane 0 writes
// its results. Returns the row status, or -1 when the row needs the block
// kernels (complexCompact of more than SORT cells: *ncells_out set, nothing
// written).
template <uint32_t SORT>
DEVI int cq_row_lds(const CompactArgs& a, uint64_t r, const RowHdr& h, const RowBufs& L, const RowLds& p,
                    uint32_t* keys, uint32_t* pay, uint32_t* runs, int lane, uint32_t* qlen_out, uint32_t* vlen_out,
                    uint32_t* ncells_out) {
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
    const uint32_t qpos = min(p.qi + qcar + qi - ql, L.qlim), vpos = min(p.vi + vcar + vi - vl, L.vlim);
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
  int reached = 0;
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
    if (ncells > SORT) {  // too many cells for the in-wave sort: block kernels
      *ncells_out = ncells;
      return -1;
    }
#ifdef CR_ABL
    if (CR_ABL & 2) st = CQ_ERROR; else
#endif
    st = cq_complex_lds<SORT>(L, p, nk, nvalid - nmulti, ncells, keys, pay, runs, lane, &oql, &ovl);
    reached = CQ_REACHED_COMPLEX;
  } else if (!any_fix && !any_junk) {
    // trivialCompact changes nothing: qualifiers and values pass through
    st = CQ_TRIVIAL;
    if (L.qout + p.qo != L.qin + p.qi)
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
      if (valid) {  // (in place: output position <= the input position of every later read)
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
  *qlen_out = oql;
  *vlen_out = ovl;
  return st | reached;
}

// ===========================================================================
// The write/delete decision of complexCompact rows
// (CompactionQueue.java:355-404). `longest` is the row's first KV as handed
// in, replaced by each later non-2-byte, even, non-empty qualifier strictly
// longer than it (:283-312); if the compacted qualifier is not longer than
// longest's, the KV holding exactly the compacted qualifier — longest itself
// if it matches, else the first such KV in row order (:369-387) — is kept
// out of the delete set, and nothing is written when its value is the
// compacted value too (:388-399). One wave per row. k_compact_rows decides
// its own rows from LDS (cq_dup_core with the compacted bytes in LDS);
// k_compact_dups takes the rows k_compact_complex finished.
// ===========================================================================
// (x: global, y: global or LDS)
DEVI bool cq_wave_equal(const uint8_t* x, const uint8_t* y, uint32_t n, int lane) {
  bool ne = false;
  for (uint32_t j = lane; j < n; j += WAVE) ne |= x[j] != y[j];
  return ballot(ne) == 0;
}

// KV lengths through ql(i) / vl(i); cq / cv: the compacted qualifier and value.
template <class QL, class VL>
DEVI void cq_dup_core(const CompactArgs& a, uint64_t r, uint64_t nk, uint64_t qs, uint64_t vs, uint32_t cql,
                      uint32_t cvl, const uint8_t* cq, const uint8_t* cv, QL qlf, VL vlf, int lane) {
  // ---- longest (:283-312) ----
  uint32_t lbest = qlf(0);
  uint64_t li = 0, lq = qs, lv = vs;
  uint32_t lvl = vlf(0);
  uint64_t qcar = 0, vcar = 0;
  for (uint64_t base = 0; base < nk; base += WAVE) {
    const uint64_t i = base + lane;
    const bool act = i < nk;
    const uint32_t ql = act ? qlf(i) : 0u, vl = act ? vlf(i) : 0u;
    const uint32_t qi = wave_incl_scan_u32_dpp(ql), vi = wave_incl_scan_u32_dpp(vl);
    const uint64_t qpos = qs + qcar + (qi - ql), vpos = vs + vcar + (vi - vl);
    qcar += readlane_u32(qi, 63);
    vcar += readlane_u32(vi, 63);
    const bool multi = act && ql != 2 && ql != 0 && (ql & 1) == 0;
    const uint32_t mx = wave_max_u32_dpp(multi ? ql : 0u);
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
      const uint32_t ql = act ? qlf(i) : 0u, vl = act ? vlf(i) : 0u;
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

DEVI void cq_dup_row(const CompactArgs& a, uint64_t r, int lane) {
  const uint64_t kb = a.row_kv_start[r], nk = a.row_kv_start[r + 1] - kb;
  cq_dup_core(
      a, r, nk, a.row_qual_off[r], a.row_val_off[r], a.out_qlen[r], a.out_vlen[r], a.oq + a.out_qoff[r],
      a.ov + a.out_voff[r], [&](uint64_t i) { return (uint32_t)a.kv_qual_len[kb + i]; },
      [&](uint64_t i) { return (uint32_t)a.kv_val_len[kb + i]; }, lane);
}

// The rows k_compact_complex finished (its two lists; k_compact_rows decides
// its own rows from LDS), a wave a listed row.
__global__ void __launch_bounds__(256) k_compact_dups(CompactArgs a) {
  const int lane = lane_id();
  const uint32_t n0 = a.counters[0], n = n0 + a.counters[1];
  for (uint32_t i = blockIdx.x * 4 + threadIdx.x / WAVE; i < n; i += gridDim.x * 4) {
    const uint32_t r = i < n0 ? a.list_lds[i] : a.list_big[i - n0];
    if (a.status[r] == CQ_COMPLEX) cq_dup_row(a, r, lane);
  }
}

// ===========================================================================
// Value output of trivially compacted rows. Row r's output (region [s, e) =
// its input value bytes + 1, placed at row_val_off[r] - V0 + r) is its input
// with the 4-byte zero prefix of each legacy float removed (the row's holes:
// output positions h, in(y) = row_val_off[r] + y + 4 * #{h <= y}), then its
// meta byte 0; the 4 * holes bytes after the meta byte are unused. Every
// aligned 16-B output chunk is written once, by the row holding its first
// byte (with the next row's head when the row ends inside it); chunks
// crossing two row ends or two holes go byte by byte.
// ===========================================================================
struct CvRow {
  uint64_t s, e, in;  // output region [s, e), input offset of the first byte
  uint32_t h0, h1;
  bool ok;
};
DEVI uint64_t cv_meta(const CvRow& w) { return w.e - 1 - 4ull * ((w.h0 != ~0u) + (w.h1 != ~0u)); }

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

struct CvLds {  // the source: a piece's value bytes in LDS
  const uint8_t* v;
  uint64_t base;  // input offset of LDS byte 0
  DEVI uint4 v16(uint64_t x) const { return lds_ld16_any(v, (uint32_t)(x - base)); }
  DEVI uint8_t b(uint64_t x) const { return v[x - base]; }
};

// One aligned 16-B output chunk c (absolute address) whose first byte lies in
// row r (w; n = row r + 1, when there is one): one source, one hole or the
// row end inside (two sources selected by byte), or byte by byte.
// (row_at(ru, u): row ru's CvRow into u, false past the piece's rows)
template <class RowAt, class Dst>
DEVI void cv_chunk_t(const CompactArgs& a, uint64_t r, const CvRow& w, const CvRow& n, uintptr_t c,
                     uintptr_t ov_abs, RowAt row_at, const CvLds& src, const Dst& dst) {
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
  if (c1 || c2) {
    const uint64_t xB = c1 ? xa + 4 : xb;
    const int pos = c1 ? (in0 ? (int)(w.h0 - y0) : in1 ? (int)(w.h1 - y0) : 16) : (int)(m - o);
    dst.put16(c, cq_funnel(src.v16(xa), src.v16(xB), pos, !c1));
  } else {  // byte by byte, walking the rows (two boundaries in the chunk)
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
      dst.put1(c + b, ob == mu ? (uint8_t)0 : src.b(u.in + y + 4 * ((u.h0 <= y) + (u.h1 <= y))));
    }
  }
}

// ===========================================================================
// Helpers of the wave kernels.
// ===========================================================================
// wave-uniform values read from LDS, moved to scalar registers
DEVI uint32_t uni32(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
DEVI uint64_t uni64(uint64_t v) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(v >> 32)) << 32) | __builtin_amdgcn_readfirstlane((uint32_t)v);
}

// Writes lds[i0 + (x - b0)] to dst[x] for x in [b0, b1): 16-B stores where a
// whole aligned chunk of dst lies inside the range (LDS read at any byte
// index), byte stores at the edges (lanes 0-15 head, 16-31 tail).
DEVI void cq_unstage_wave(uint8_t* dst, const uint8_t* lds, uint32_t i0, uint64_t b0, uint64_t b1, int lane) {
  if (b1 <= b0) return;
  const uintptr_t s = (uintptr_t)(dst + b0), e = (uintptr_t)(dst + b1);
  const uintptr_t a0 = (s + 15) & ~(uintptr_t)15, a1 = e & ~(uintptr_t)15;  // whole chunks [a0, a1)
  for (uintptr_t cs = a0 + 16ull * lane; cs < a1; cs += 16ull * WAVE)
    *(uint4*)cs = lds_ld16_any(lds, i0 + (uint32_t)(cs - s));
  const uintptr_t h1 = a0 < e ? a0 : e;
  const uintptr_t t0 = a1 > h1 ? a1 : h1;
  uintptr_t x = 0;
  if (lane < 16) x = s + lane;
  else if (lane < 32) x = t0 + (lane - 16);
  if ((lane < 16 && x < h1) || (lane >= 16 && lane < 32 && x < e)) *(uint8_t*)x = lds[i0 + (uint32_t)(x - s)];
}

// ===========================================================================
// k_compact_rows: every row k_compact_wave left CQ_PENDING (not plain: single
// KVs, junk, errors, complexCompact, more than two legacy floats; or over its
// budget). A block takes a range of CR_RANGE rows, gathers its pending rows
// (ballots over the statuses, one barrier), and each wave then takes rows of
// that list on its own: the row's KV lengths, qualifier and value bytes
// staged into the wave's LDS (16-B loads, all in flight), cq_row_lds (the
// compacted qualifier over its input, the value into an output slot at the
// destination's 16-B phase), the write/delete decision from the same LDS,
// the row's output written with 16-B stores inside it. Wave-level LDS syncs
// only. Rows over the wave's budget go through cq_row_global; complex rows of
// more than CW_SORT cells to the k_compact_complex lists.
// ===========================================================================
#ifndef CR_RANGE
#define CR_RANGE 256u   // rows scanned for CQ_PENDING per block iteration
#endif
#ifndef CR_WAVES
#define CR_WAVES 4u     // waves a block (C5 call: 4 waves / 256 rows 0.802 ms, 2 / 128 0.805, 1 / 64 0.807, 2 / 256 0.856, 1 / 128 0.848)
#endif
#ifndef CR_KCAP
#define CR_KCAP 256u    // a row in LDS: KVs
#endif
#ifndef CR_QCAP
#define CR_QCAP 1024u   // qualifier bytes
#endif
#ifndef CR_VCAP
#define CR_VCAP 2048u   // value bytes
#endif
#ifndef CW_SORT
#define CW_SORT 128u    // cells of an in-wave complexCompact
#endif
#ifndef CR_WPE
#define CR_WPE 5        // waves per SIMD the register allocation aims at (the compiler's 119 VGPRs; 5: -0.02 ms, 6: none)
#endif
#ifndef CR_ABL
#define CR_ABL 0        // (ablation builds only, wrong results: 1 no write/delete decision, 2 no complexCompact)
#endif
static_assert(CW_SORT % WAVE == 0 && (CW_SORT & (CW_SORT - 1)) == 0, "in-wave sort size");
struct __attribute__((aligned(16))) CrLds {
  uint8_t qlen[2 * CR_KCAP + 32];
  uint8_t vlen[2 * CR_KCAP + 32];
  uint8_t qin[CR_QCAP + 32];   // (the compacted qualifier is written over it)
  uint8_t vin[CR_VCAP + 32];
  uint8_t vout[CR_VCAP + 48];  // (at the destination's 16-B phase)
  uint32_t keys[CW_SORT], pay[CW_SORT], runs[CQ_RUNS_SLOTS];
};

// the headers of up to 10 rows, six words a row (lanes 6 m .. 6 m + 5:
// row_kv_start, row_qual_off, row_val_off at r and r + 1), in one round trip
DEVI uint64_t cr_hdr_load(const CompactArgs& a, const uint32_t* list, uint32_t i0, uint32_t step, uint32_t n,
                          int lane) {
  const uint32_t m = (uint32_t)lane / 6, f = (uint32_t)lane % 6, i = i0 + step * m;
  if (m >= 10 || i >= n) return 0ull;
  const uint32_t r = list[i];
  const uint64_t* p = f < 2 ? a.row_kv_start : f < 4 ? a.row_qual_off : a.row_val_off;
  return p[r + (f & 1)];
}
// (cq_row's header from row m's six words)
DEVI RowHdr cr_hdr(const CompactArgs& a, uint64_t v, uint32_t m, uint64_t r, uint64_t Q0, uint64_t V0) {
  RowHdr h;
  h.kb = readlane_u64(v, 6 * m);
  const uint64_t ke = readlane_u64(v, 6 * m + 1);
  h.qs = readlane_u64(v, 6 * m + 2);
  h.qe = readlane_u64(v, 6 * m + 3);
  h.vs = readlane_u64(v, 6 * m + 4);
  h.ve = readlane_u64(v, 6 * m + 5);
  h.ok = h.kb <= ke && ke <= a.n_kvs && h.qs <= h.qe && h.qe <= a.qual_nbytes && h.vs <= h.ve &&
         h.ve <= a.val_nbytes && h.qs >= Q0 && h.vs >= V0 && (h.ve - h.vs) < (1ull << 32);
  h.nk = h.ok ? ke - h.kb : 0;
  h.oqo = h.qs - Q0;
  h.ovo = h.vs - V0 + r;
  h.ok = h.ok && h.oqo + (h.qe - h.qs) <= a.qcap && h.ovo + (h.ve - h.vs) + 1 <= a.vcap;
  return h;
}

DEVI void cr_row(const CompactArgs& a, CrLds& L, const RowHdr& h, uint64_t r, uint32_t* n_cx, int lane) {
  if (lane == 0) {
    a.out_qoff[r] = h.oqo;
    a.out_voff[r] = h.ovo;
  }
  if (!h.ok || h.nk > CR_KCAP || h.qe - h.qs > CR_QCAP || h.ve - h.vs > CR_VCAP) {
    cq_row_global(a, r, lane);
    return;
  }
  // ---- staging: the four segments' 16-B chunks in one flat loop (every
  // load of the row in flight together) ----
  const uintptr_t sk = (uintptr_t)(a.kv_qual_len + h.kb), sv = (uintptr_t)(a.kv_val_len + h.kb);
  const uintptr_t sq = (uintptr_t)(a.qual + h.qs), sx = (uintptr_t)(a.val + h.vs);
  const uint32_t hk = (uint32_t)(sk & 15u), hv = (uint32_t)(sv & 15u), hq = (uint32_t)(sq & 15u), hx = (uint32_t)(sx & 15u);
  const uint32_t nk = (uint32_t)h.nk;
  const uint32_t n1 = nk ? (hk + 2 * nk + 15) / 16 : 0u, n2 = n1 + (nk ? (hv + 2 * nk + 15) / 16 : 0u);
  const uint32_t n3 = n2 + (h.qe > h.qs ? (uint32_t)((hq + (h.qe - h.qs) + 15) / 16) : 0u);
  const uint32_t n4 = n3 + (h.ve > h.vs ? (uint32_t)((hx + (h.ve - h.vs) + 15) / 16) : 0u);
  auto at = [&](uint32_t c, uint4*& d) {
    if (c < n1) { d = (uint4*)L.qlen + c; return (const uint4*)(sk - hk) + c; }
    if (c < n2) { d = (uint4*)L.vlen + (c - n1); return (const uint4*)(sv - hv) + (c - n1); }
    if (c < n3) { d = (uint4*)L.qin + (c - n2); return (const uint4*)(sq - hq) + (c - n2); }
    d = (uint4*)L.vin + (c - n3);
    return (const uint4*)(sx - hx) + (c - n3);
  };
  for (uint32_t c = lane; c < n4; c += 2 * WAVE) {
    const bool b = c + WAVE < n4;
    uint4 *d0, *d1 = nullptr;
    const uint4* g0 = at(c, d0);
    const uint4* g1 = b ? at(c + WAVE, d1) : nullptr;
    const uint4 v0 = *g0;
    uint4 v1 = {};
    if (b) v1 = *g1;
    *d0 = v0;
    if (b) *d1 = v1;
  }
  RowLds p;
  p.k0 = hk;
  p.kv0 = hv;
  p.qi = p.qo = hq;
  p.vi = hx;
  p.vo = (uint32_t)((uintptr_t)(a.ov + h.ovo) & 15u);
  wave_lds_sync();
  const RowBufs B{L.qlen, L.vlen, L.qin, L.vin, L.qin, L.vout, CR_QCAP + 14, CR_VCAP + 14};
  uint32_t oql = 0, ovl = 0, nc = 0;
  const int st = cq_row_lds<CW_SORT>(a, r, h, B, p, L.keys, L.pay, L.runs, lane, &oql, &ovl, &nc);
  if (st < 0) {  // complexCompact of more cells than the wave sorts: k_compact_complex
    if (lane == 0) {
      if (nc <= CQ_LDS_CELLS) a.list_lds[atomicAdd(&a.counters[0], 1u)] = (uint32_t)r;
      else a.list_big[atomicAdd(&a.counters[1], 1u)] = (uint32_t)r;
    }
    return;
  }
  wave_lds_sync();
  if (st & CQ_REACHED_COMPLEX) {
    (*n_cx)++;
    if ((st & 0xFF) == CQ_COMPLEX && a.out_write && !(CR_ABL & 1))
      cq_dup_core(
          a, r, h.nk, h.qs, h.vs, oql, ovl, L.qin + p.qo, L.vout + p.vo,
          [&](uint64_t k) { return lds_u16(L.qlen, p.k0 + 2 * (uint32_t)k); },
          [&](uint64_t k) { return lds_u16(L.vlen, p.kv0 + 2 * (uint32_t)k); }, lane);
  }
  cq_unstage_wave(a.oq, L.qin, p.qo, h.oqo, h.oqo + oql, lane);
  cq_unstage_wave(a.ov, L.vout, p.vo, h.ovo, h.ovo + ovl, lane);
  wave_lds_sync();  // (the row's LDS consumed before the wave's next row is staged)
}

__global__ void __launch_bounds__(WAVE * CR_WAVES)
#if CR_WPE
__attribute__((amdgpu_waves_per_eu(CR_WPE, CR_WPE)))
#endif
k_compact_rows(CompactArgs a) {
  constexpr uint32_t NW = CR_WAVES;
  static_assert(CR_RANGE % NW == 0 && CR_RANGE / NW >= 1, "rows kernel range");
  __shared__ CrLds Ls[NW];
  __shared__ uint32_t s_list[CR_RANGE], s_wn[NW], s_cx;
  const int tid = threadIdx.x, lane = lane_id(), w = tid / WAVE;
  const uint64_t Q0 = a.row_qual_off[0], V0 = a.row_val_off[0];
  if (tid == 0) s_cx = 0;
  uint32_t n_cx = 0;
  for (uint64_t rb = (uint64_t)blockIdx.x * CR_RANGE; rb < a.n_rows; rb += (uint64_t)gridDim.x * CR_RANGE) {
    // ---- the range's CQ_PENDING rows, in row order, into s_list ----
    __syncthreads();  // (the previous range's list consumed)
    constexpr uint32_t QR = CR_RANGE / NW;  // a wave's share of the range
    constexpr int CR_U = (int)((QR + WAVE - 1) / WAVE);
    uint32_t pend[CR_U], wpos = 0;
#pragma unroll
    for (int u = 0; u < CR_U; u++) {
      const uint32_t q = u * WAVE + lane;  // (wave w: its share of the range)
      const uint64_t r = rb + (uint64_t)w * QR + q;
      const bool pd = q < QR && r < a.n_rows && a.status[r] == CQ_PENDING;
      const uint64_t m = ballot(pd);
      pend[u] = pd ? wpos + (uint32_t)__popcll(m & lanemask_lt(lane)) : ~0u;
      wpos += (uint32_t)__popcll(m);
    }
    if (lane == 0) s_wn[w] = wpos;
    __syncthreads();
    uint32_t woff = 0;
    for (int v = 0; v < w; v++) woff += s_wn[v];
    uint32_t n = 0;
    for (uint32_t v = 0; v < NW; v++) n += s_wn[v];
#pragma unroll
    for (int u = 0; u < CR_U; u++)
      if (pend[u] != ~0u) s_list[woff + pend[u]] = (uint32_t)(rb + (uint64_t)w * QR + u * WAVE + lane);
    __syncthreads();
    // ---- a wave a row; its rows' headers loaded ten at a time ----
    for (uint32_t i0 = w; i0 < n; i0 += 10 * NW) {
      const uint64_t hv = cr_hdr_load(a, s_list, i0, NW, n, lane);
      for (uint32_t m = 0; m < 10 && i0 + NW * m < n; m++) {
        const uint32_t r = uni32(s_list[i0 + NW * m]);
        cr_row(a, Ls[w], cr_hdr(a, hv, m, r, Q0, V0), r, &n_cx, lane);
      }
    }
  }
  if (lane == 0 && n_cx) atomicAdd(&s_cx, n_cx);
  __syncthreads();
  if (tid == 0 && s_cx) atomicAdd(&a.counters[3], s_cx);
}

// ===========================================================================
// k_compact_wave: the plain rows of a batch, one wave per run of CW_ROWS
// consecutive rows (round 6; replaces the block-wide k_compact_plain, whose
// chain of ~8 block barriers per run left each CU with 2 runs in flight). A
// row is plain when it holds >= 2 KVs, every qualifier is 2 bytes, every value
// 1..8 bytes, legacy floats are fixable (at most two a row) and the time
// deltas strictly increase in KV order: trivialCompact's output is then the
// row's qualifier and value bytes with two local fix-ups, plus the 0 meta
// byte (CompactionQueue.java:286-351, 450-474, fixes :490-544). A run is cut
// into pieces whose KV lengths, qualifier and value bytes fit the wave's LDS;
// per piece:
//   1. staging: the KV lengths, qualifier and value bytes, 16-B loads, all in
//      flight together (one round trip);
//   2. the plain test flat over the piece's KVs, CW_KPT consecutive KVs a
//      lane, each KV's row by comparing with the rows' first KVs: value
//      offsets and legacy-float counts inside each row from one wave scan,
//      the flag fix-ups patched in LDS (fixQualifierFlags :490-499), the
//      first two legacy floats' output positions (fixFloatingPointValue
//      drops their 4-byte zero prefix, :510-544);
//   3. plain rows' results (status TRIVIAL, lengths, write decision), the
//      others CQ_PENDING (k_compact_rows);
//   4. the piece's qualifiers and values written with 16-B stores from LDS:
//      the values of every row as if plain (cv_chunk_t: shifted by its index
//      around its holes, then its meta byte) — a pending row's range is
//      rewritten by k_compact_rows; byte stores only at the piece's two
//      edges, so no byte has two writers in this kernel.
// A run with offsets out of bounds and a row over the piece budget alone are
// left CQ_PENDING. Wave-level LDS syncs only (wave_lds_sync): the CU's
// resident waves never wait for each other, so they overlap each other's
// staging, tests and stores.
// ===========================================================================
#ifndef CW_ROWS
#define CW_ROWS 4u     // rows per wave run
#endif
#ifndef CW_KCAP
#define CW_KCAP 256u   // KVs per piece
#endif
#ifndef CW_QCAP
#define CW_QCAP 768u   // qualifier bytes per piece
#endif
#ifndef CW_VCAP
#define CW_VCAP 1536u  // value bytes per piece
#endif
#ifndef CW_WAVES
#define CW_WAVES 2u    // waves a block (C5 call, same box: 1 / 2 / 4 / 8 waves 0.794 / 0.798 / 0.845 / 0.925 ms: a block frees its slot only when its last wave ends)
#endif
#ifndef CW_WPE
#define CW_WPE 7       // waves per SIMD the register allocation aims at (C5 call, same box: the compiler's 80 VGPRs 0.898 ms, 7: 0.856, 8: 0.956)
#endif
#ifndef CW_ABL
#define CW_ABL 0       // (ablation builds only, wrong results: 2 no value output, 4 no plain test)
#endif
constexpr uint32_t CW_KPT = CW_KCAP / WAVE;  // KVs a lane
static_assert(CW_KPT == 4 || CW_KPT == 8, "k_compact_wave: 4 or 8 KVs a lane");
static_assert(CW_ROWS >= 1 && CW_ROWS < WAVE, "k_compact_wave: rows a run");
// the staged piece: four segments back to back in 16-B chunk order (the KV
// qualifier lengths, the KV value lengths, the qualifier bytes, the value
// bytes; each from its source's aligned 16-B chunk holding the piece's first
// byte)
constexpr uint32_t CW_CHUNKS = 2 * ((14 + 2 * CW_KCAP + 15) / 16) + (15 + CW_QCAP + 15) / 16 + (15 + CW_VCAP + 15) / 16;
struct __attribute__((aligned(16))) CwLds {
  uint8_t pad0[16];                  // (cv_chunk's second source may start one byte before the piece's values)
  uint8_t buf[16 * CW_CHUNKS + 16];  // (lds_ld16_any reads up to 4 bytes past its 16)
  uint64_t kv[CW_ROWS + 1], qo[CW_ROWS + 1], vo[CW_ROWS + 1];  // the run's row offsets
  CvRow w[CW_ROWS];
  // the piece's rows (index i = row - j0): first KV (relative) | plain
  // candidate (>= 2 KVs, 2 qualifier bytes each) << 31, LDS index of the
  // first qualifier byte, value bytes, first value byte (relative)
  uint4 rec[CW_ROWS];
  uint32_t pstart[CW_ROWS], pend[CW_ROWS];  // scan prefix (value bytes | legacy floats << 16) around the row's KVs
  uint32_t bad[CW_ROWS], h0[CW_ROWS], h1[CW_ROWS];
};
struct CvGlobalDst {  // cv_chunk_t's destination: the output value bytes
  DEVI void put16(uintptr_t c, const uint4& x) const { *(uint4*)c = x; }
  DEVI void put1(uintptr_t c, uint8_t x) const { *(uint8_t*)c = x; }
};

// One piece [j0, j1) of the run starting at row r0.
DEVI void cw_piece(const CompactArgs& a, CwLds& L, uint64_t r0, uint32_t j0, uint32_t j1, uint64_t Q0, uint64_t V0) {
  const uint32_t t = lane_id(), np = j1 - j0;
  const uint64_t KA = uni64(L.kv[j0]), QA = uni64(L.qo[j0]), QB = uni64(L.qo[j1]), VA = uni64(L.vo[j0]);
  const uint64_t VB = uni64(L.vo[j1]);
  const uint32_t NK = uni32((uint32_t)(L.kv[j1] - KA));
  // ---- 1. staging ----
  const uintptr_t sk = (uintptr_t)(a.kv_qual_len + KA), sv = (uintptr_t)(a.kv_val_len + KA), sq = (uintptr_t)(a.qual + QA);
  const uintptr_t sx = (uintptr_t)(a.val + VA);
  const uint32_t hkb = (uint32_t)(sk & 15u), hvb = (uint32_t)(sv & 15u), hq = (uint32_t)(sq & 15u);
  const uint32_t hx = (uint32_t)(sx & 15u);
  const uint32_t nk1 = NK ? (hkb + 2 * NK + 15) / 16 : 0u, nv1 = NK ? (hvb + 2 * NK + 15) / 16 : 0u;
  const uint32_t nq1 = QB > QA ? (uint32_t)((hq + (QB - QA) + 15) / 16) : 0u;
  const uint32_t nx1 = VB > VA ? (uint32_t)((hx + (VB - VA) + 15) / 16) : 0u;
  const uint32_t e1 = nk1 + nv1, e2 = e1 + nq1, tot = e2 + nx1;
  auto src = [&](uint32_t c) {
    return c < nk1  ? (const uint4*)(sk - hkb) + c
           : c < e1 ? (const uint4*)(sv - hvb) + (c - nk1)
           : c < e2 ? (const uint4*)(sq - hq) + (c - e1)
                    : (const uint4*)(sx - hx) + (c - e2);
  };
  uint4* const dst = (uint4*)L.buf;
  for (uint32_t c = t; c < tot; c += 4 * WAVE) {  // (four named register sets: an array lands in scratch)
    const bool b1 = c + WAVE < tot, b2 = c + 2 * WAVE < tot, b3 = c + 3 * WAVE < tot;
    const uint4 v0 = *src(c);
    uint4 v1 = {}, v2 = {}, v3 = {};
    if (b1) v1 = *src(c + WAVE);
    if (b2) v2 = *src(c + 2 * WAVE);
    if (b3) v3 = *src(c + 3 * WAVE);
    dst[c] = v0;
    if (b1) dst[c + WAVE] = v1;
    if (b2) dst[c + 2 * WAVE] = v2;
    if (b3) dst[c + 3 * WAVE] = v3;
  }
  const uint8_t* const Bql = L.buf + hkb;             // KV qualifier lengths
  const uint8_t* const Bvl = L.buf + 16 * nk1 + hvb;  // KV value lengths
  uint8_t* const Bq = L.buf + 16 * e1;                // qualifier bytes (index: offset - QA + hq)
  const uint8_t* const Bx = L.buf + 16 * e2 + hx;     // value bytes (index: offset - VA)
  if (t < np) {  // the piece's rows
    const uint32_t j = j0 + t;
    const uint64_t nk = L.kv[j + 1] - L.kv[j];
    const uint32_t k0 = (uint32_t)(L.kv[j] - KA);
    const bool cand = nk >= 2 && L.qo[j + 1] - L.qo[j] == 2 * nk;
    L.rec[t] = make_uint4(k0 | (cand ? 1u << 31 : 0u), (uint32_t)(L.qo[j] - QA) + hq, (uint32_t)(L.vo[j + 1] - L.vo[j]),
                          (uint32_t)(L.vo[j] - VA));
    L.pstart[t] = L.pend[t] = 0;
    L.bad[t] = 0;
    L.h0[t] = L.h1[t] = ~0u;
  }
  // the rows' first KVs (uniform): KV k's row is the number of them <= k
  uint32_t ks[CW_ROWS];
#pragma unroll
  for (int i = 1; i < (int)CW_ROWS; i++) ks[i] = (uint32_t)i < np ? uni32((uint32_t)(L.kv[j0 + i] - KA)) : 0xFFFFFFFFu;
  wave_lds_sync();
  // ---- 2. the plain test, flat over the KVs: CW_KPT consecutive KVs a lane ----
  const uint32_t kb = CW_KPT * t;
  const bool any = kb < NK && !(CW_ABL & 4);
  uint32_t ir[CW_KPT], q_[CW_KPT], ql_[CW_KPT], vl_[CW_KPT], c_[CW_KPT], pre_[CW_KPT];
  uint32_t fm = 0, lm = 0;  // bit u: KV kb + u is its row's first / last
  uint32_t sum = 0;
  {
    uint4 ql4[(CW_KPT + 7) / 8] = {}, vl4[(CW_KPT + 7) / 8] = {};
    if (any) {
#pragma unroll
      for (int w = 0; w < (int)((CW_KPT + 7) / 8); w++) {
        ql4[w] = lds_ld16_any(Bql, 2 * kb + 16 * w);
        vl4[w] = lds_ld16_any(Bvl, 2 * kb + 16 * w);
      }
    }
#pragma unroll
    for (int u = 0; u < (int)CW_KPT; u++) {
      const uint32_t k = kb + u;
      const bool act = any && k < NK;
      const uint32_t qw = u % 8 < 2 ? ql4[u / 8].x : u % 8 < 4 ? ql4[u / 8].y : u % 8 < 6 ? ql4[u / 8].z : ql4[u / 8].w;
      const uint32_t vw = u % 8 < 2 ? vl4[u / 8].x : u % 8 < 4 ? vl4[u / 8].y : u % 8 < 6 ? vl4[u / 8].z : vl4[u / 8].w;
      uint32_t row = 0;
      bool first = k == 0, last = k + 1 >= NK;
#pragma unroll
      for (int i = 1; i < (int)CW_ROWS; i++) {
        row += k >= ks[i] ? 1u : 0u;
        first |= k == ks[i];
        last |= k + 1 == ks[i];
      }
      ir[u] = row;
      if (act && first) fm |= 1u << u;
      if (act && last) lm |= 1u << u;
      ql_[u] = act ? (qw >> (16 * (u % 2))) & 0xFFFFu : 0u;
      vl_[u] = act ? (vw >> (16 * (u % 2))) & 0xFFFFu : 0u;
      q_[u] = 0;
      c_[u] = 0;
      if (act) {
        const uint4 R = L.rec[row];
        if ((R.x >> 31) && ql_[u] == 2) q_[u] = lds_q16(Bq, R.y + 2 * (k - (R.x & 0x7FFFFFFFu)));
        const bool leg = (R.x >> 31) && ql_[u] == 2 && cq_legacy(q_[u] & 0xFFu, vl_[u]);  // :510-515
        c_[u] = min(vl_[u], 9u) | (leg ? 1u << 16 : 0u);
      }
      pre_[u] = sum;  // (exclusive, inside the lane)
      sum += c_[u];
    }
  }
  const uint32_t ex = wave_incl_scan_u32_dpp(sum) - sum;
  // each row's scan prefix before its first KV and after its last, by the
  // lanes owning those KVs (a row without KVs is not plain: never read)
#pragma unroll
  for (int u = 0; u < (int)CW_KPT; u++) {
    if (fm & (1u << u)) L.pstart[ir[u]] = ex + pre_[u];
    if (lm & (1u << u)) L.pend[ir[u]] = ex + pre_[u] + c_[u];
  }
  wave_lds_sync();
  if (any) {
#pragma unroll
    for (int u = 0; u < (int)CW_KPT; u++) {
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
        const uint32_t qp = u > 0 ? q_[u > 0 ? u - 1 : 0] : lds_q16(Bq, qpos - 2);
        kbad = (q >> 4) <= (qp >> 4);
      }
      if (!kbad) kbad = vin + vl > R.z;
      if (leg && !kbad) {  // the 4-byte zero prefix (fixFloatingPointValue :530-544)
        const uint8_t* vp = Bx + R.w + vin;
        kbad = (vp[0] | vp[1] | vp[2] | vp[3]) != 0;
      }
      if (!kbad) {  // fixQualifierFlags :490-499 (delta bits unchanged: a neighbour's order check
                    // reads the same delta before or after the patch)
        const uint8_t f = (uint8_t)cq_fixq(q & 0xFFu, leg ? 4u : vl);
        if (f != (uint8_t)q) Bq[qpos + 1] = f;
      } else {
        L.bad[i] = 1;
      }
      if (leg) {  // the holes: output positions of the row's first two legacy floats
        if (nl == 0) L.h0[i] = vin;
        else if (nl == 1) L.h1[i] = vin - 4;
      }
    }
  }
  wave_lds_sync();
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
      a.status[r] = CQ_PENDING;  // (to k_compact_rows)
    }
  }
  wave_lds_sync();
  // ---- 4. qualifiers from LDS, values around the holes ----
  {
    const uintptr_t q0 = (uintptr_t)a.oq + (QA - Q0), q1 = (uintptr_t)a.oq + (QB - Q0);
    const uintptr_t qc0 = (q0 + 15) & ~(uintptr_t)15, qc1 = q1 & ~(uintptr_t)15;
    for (uintptr_t c = qc0 + 16ull * t; c < qc1; c += 16ull * WAVE) *(uint4*)c = lds_ld16_any(Bq, (uint32_t)(c - q0) + hq);
    const uintptr_t he = qc0 < q1 ? qc0 : q1, ts = qc1 > he ? qc1 : he;  // edge bytes [q0, he), [ts, q1)
    const uintptr_t x = t < 16 ? q0 + t : ts + (t - 16);
    if ((t < 16 && x < he) || (t >= 16 && t < 32 && x < q1)) *(uint8_t*)x = Bq[(uint32_t)(x - q0) + hq];
  }
  {
    const uintptr_t ov_abs = (uintptr_t)a.ov;
    const uintptr_t d0 = ov_abs + uni64(L.w[0].s), d1 = ov_abs + uni64(L.w[np - 1].e);
    const uintptr_t c0 = (d0 + 15) & ~(uintptr_t)15, c1 = d1 & ~(uintptr_t)15;
    const CvLds xs{L.pad0, VA - 16 - 16 * e2 - hx};
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
    for (uintptr_t c = c0 + 16ull * t; c < c1 && !(CW_ABL & 2); c += 16ull * WAVE) {
      const uint32_t i = find(c - ov_abs);
      CvRow n = {};
      if (i + 1 < np) n = L.w[i + 1];
      cv_chunk_t(a, r0 + j0 + i, L.w[i], n, c, ov_abs, row_at, xs, CvGlobalDst{});
    }
    const uintptr_t he = c0 < d1 ? c0 : d1, ts = c1 > he ? c1 : he;  // edge bytes [d0, he), [ts, d1)
    const uintptr_t x = t < 16 ? d0 + t : ts + (t - 16);
    if ((t < 16 && x < he) || (t >= 16 && t < 32 && x < d1)) {
      const uint64_t o = x - ov_abs;
      const CvRow& u = L.w[find(o)];
      const uint64_t m = cv_meta(u), y = o - u.s;
      if (o <= m) *(uint8_t*)x = o == m ? (uint8_t)0 : xs.b(u.in + y + 4 * ((u.h0 <= y) + (u.h1 <= y)));
    }
  }
}

__global__ void __launch_bounds__(WAVE * CW_WAVES)
#if CW_WPE
__attribute__((amdgpu_waves_per_eu(CW_WPE, CW_WPE)))
#endif
k_compact_wave(CompactArgs a) {
  __shared__ CwLds Ls[CW_WAVES];
  const uint32_t t = lane_id();
  CwLds& L = Ls[threadIdx.x / WAVE];
  const uint64_t r0 = ((uint64_t)blockIdx.x * CW_WAVES + threadIdx.x / WAVE) * CW_ROWS;
  if (r0 >= a.n_rows) return;
  const uint32_t nr = (uint32_t)min((uint64_t)CW_ROWS, a.n_rows - r0);
  const uint64_t Q0 = a.row_qual_off[0], V0 = a.row_val_off[0];
  if (r0 == 0 && t == 0 && a.ext_out) {  // (the batch's extents, for the host's checks at the call's end)
    a.ext_out[0] = Q0;
    a.ext_out[1] = a.row_qual_off[a.n_rows];
    a.ext_out[2] = V0;
    a.ext_out[3] = a.row_val_off[a.n_rows];
  }
  if (t <= nr) {
    L.kv[t] = a.row_kv_start[r0 + t];
    L.qo[t] = a.row_qual_off[r0 + t];
    L.vo[t] = a.row_val_off[r0 + t];
  }
  wave_lds_sync();
  bool insane = false;
  if (t < nr) {  // the row's offsets in bounds (then its ranges are disjoint from every other row's)
    const uint64_t r = r0 + t;
    const uint64_t kv = L.kv[t], kv_n = L.kv[t + 1], qo = L.qo[t], qo_n = L.qo[t + 1], vo = L.vo[t], vo_n = L.vo[t + 1];
    insane = !(kv_n >= kv && kv_n <= a.n_kvs && qo_n >= qo && vo_n >= vo && qo >= Q0 && vo >= V0 &&
               qo_n <= a.qual_nbytes && vo_n <= a.val_nbytes && qo_n - Q0 <= a.qcap && vo_n - V0 + r + 1 <= a.vcap &&
               vo_n - vo < (1ull << 32));
  }
  if (ballot(insane)) {  // the whole run to the row kernel (which finds the bad offsets)
    if (t < nr) a.status[r0 + t] = CQ_PENDING;
    return;
  }
  uint32_t j0 = 0;
  while (j0 < nr) {  // (uniform)
    uint32_t lo = j0, hi = nr;  // the most rows from j0 whose KVs and bytes fit
    while (lo < hi) {
      const uint32_t mid = (lo + hi + 1) >> 1;
      if (L.kv[mid] - L.kv[j0] <= CW_KCAP && L.qo[mid] - L.qo[j0] <= CW_QCAP && L.vo[mid] - L.vo[j0] <= CW_VCAP)
        lo = mid;
      else
        hi = mid - 1;
    }
    if (lo == j0) {  // one row over the budget alone
      if (t == 0) a.status[r0 + j0] = CQ_PENDING;
      j0++;
      continue;
    }
    cw_piece(a, L, r0, j0, lo, Q0, V0);
    j0 = lo;
    wave_lds_sync();  // (the piece's LDS consumed before the next one is staged)
  }
}
}  // namespace tsdb
