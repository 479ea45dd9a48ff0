// k_decode_fast.hip — the HBM-streaming decode(+downsample) kernel for spans
// whose rows have one value width (8-byte longs / doubles, 4-byte floats /
// ints): the reference's write paths produce exactly these rows
// (IncomingDataPoints.java:273-282, TSDB.java:285,321). Same semantics as
// k_decode.hip (RowSeq.Iterator + Span.DownsamplingIterator); any span that
// breaks the preconditions (mixed widths, dropped rows, quirk Q1, the short
// overflow, unaligned rows) is queued for the general per-span kernel.
//
// Per wave-iteration a chunk of 256 cells of one row: lane l owns cells
// 4l..4l+3 (8-byte qualifier load, 16/32-byte value loads), and the next
// chunk's loads are issued before the current one is processed.
//
// Downsampling (Span.java:377-422). Greedy bucket heads: the kernel guesses
// that buckets keep the length k of the previous one (regular cadence) and
// verifies every guessed head in parallel — head g is exact iff
// ts[g] >= end(prev) and ts[g-1] < end(prev), and the chunk tail must stay
// inside the last bucket; any mismatch reruns the chunk's heads with the
// serial ballot chain. Bucket count / timestamp sum / float count / integer
// sum are differences of DPP-scanned chunk prefix sums staged in LDS (exact
// integers); order-dependent parts (double sums of float buckets, min/max,
// dev) run one lane per bucket over the LDS-staged values in point order
// (exact). The open bucket is carried in LDS by the lane that owns it.
#pragma once
#include "dev_common.h"
#include "k_decode.hip"

namespace tsdb {

#define FCH 256  // cells per chunk

// Open/closed bucket state. The timestamp sum is kept relative to the
// bucket's first timestamp so the final floor(sum/n) is a 32-bit division.
struct FBucket {
  uint32_t n, nflt;
  int64_t ref;     // first ts of the bucket
  uint64_t rel;    // sum of (ts - ref)
  int64_t ia;      // int path: sum / min / max
  double dsum, dmm;
  Welford wf;
};

struct alignas(16) FastLds {
  uint64_t pv[FCH];   // inclusive prefix of integer values (wrapping)
  int64_t bits[FCH];  // decoded value bits (ordered pass)
  uint32_t pt[FCH];   // inclusive prefix of ts deltas within the row
  uint32_t pf[FCH];   // inclusive prefix of float cells
  uint32_t dtv[FCH];  // ts delta (qualifier >> 4) per cell
  uint8_t flt[FCH];
  uint16_t heads[FCH + 4];
  FBucket carry;      // the open bucket between chunks
};

struct RowMeta {
  uint64_t qoff, voff;
  uint32_t base, nc, w;
  bool ok;
};

DEVI RowMeta row_meta(const DecodeArgs& a, uint64_t r, const uint32_t* ncells, const uint32_t* vlen) {
  RowMeta m;
  m.qoff = a.row_qual_off[r];
  m.voff = a.row_val_off[r];
  m.base = a.row_base[r];
  m.nc = ncells[r];
  const uint32_t vl = vlen[r];
  const uint32_t vb = m.nc > 1 ? vl - 1 : vl;
  m.w = m.nc ? vb / m.nc : 0;
  m.ok = m.nc > 0 && vb == m.w * m.nc && (m.w == 8 || m.w == 4) && (m.qoff & 7) == 0 &&
         (m.voff & (m.w == 8 ? 7 : 3)) == 0 && a.row_ok[r] != 0;
  return m;
}

struct ChunkRaw {
  uint32_t q0, q1;        // 4 big-endian qualifiers (8 bytes)
  uint32_t v[8];          // 4 values (raw little-endian words)
};

DEVI void load_chunk(const DecodeArgs& a, const RowMeta& m, uint32_t c0, ChunkRaw& x) {
  const int lane = lane_id();
  const uint32_t c = c0 + 4 * lane;
  x.q0 = x.q1 = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x.v[i] = 0;
  if (c < m.nc) {
    const uint2 q = *(const uint2*)(a.qual + m.qoff + 2ull * c);
    x.q0 = q.x;
    x.q1 = q.y;
    if (m.w == 8) {
      const uint8_t* p = a.val + m.voff + 8ull * c;
      if ((m.voff & 15) == 0) {
        const uint4 u0 = *(const uint4*)p, u1 = *(const uint4*)(p + 16);
        x.v[0] = u0.x; x.v[1] = u0.y; x.v[2] = u0.z; x.v[3] = u0.w;
        x.v[4] = u1.x; x.v[5] = u1.y; x.v[6] = u1.z; x.v[7] = u1.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint2 u = *(const uint2*)(p + 8 * j);
          x.v[2 * j] = u.x; x.v[2 * j + 1] = u.y;
        }
      }
    } else {
      const uint8_t* p = a.val + m.voff + 4ull * c;
      if ((m.voff & 15) == 0) {
        const uint4 u = *(const uint4*)p;
        x.v[0] = u.x; x.v[1] = u.y; x.v[2] = u.z; x.v[3] = u.w;
      } else {
#pragma unroll
        for (int j = 0; j < 4; j++) x.v[j] = *(const uint32_t*)(p + 4 * j);
      }
    }
  }
}

// qualifier j (0..3) of this lane, host order
DEVI uint32_t qual_j(const ChunkRaw& x, int j) {
  const uint32_t word = j < 2 ? x.q0 : x.q1;
  const uint32_t h = (j & 1) ? (word >> 16) : (word & 0xFFFF);
  return ((h & 0xFF) << 8) | (h >> 8);
}

DEVI int64_t value_j(const ChunkRaw& x, int j, uint32_t w, bool flt) {
  if (w == 8) {
    const uint64_t raw = (uint64_t)x.v[2 * j] | ((uint64_t)x.v[2 * j + 1] << 32);
    return (int64_t)bswap64(raw);  // long or raw double bits
  }
  const uint32_t u = bswap32(x.v[j]);
  if (flt) return dbits((double)__uint_as_float(u));
  return (int64_t)(int32_t)u;
}

template <int AGG>
DEVI void fpush(FBucket& b, int64_t bits, bool flt, bool first) {
  const double xd = to_double(bits, flt);
  if (first) { b.dsum = xd; b.dmm = xd; if (AGG == 1 || AGG == 2) b.ia = bits; }
  else {
    b.dsum += xd;
    if (AGG == 1) { if (xd < b.dmm) b.dmm = xd; if (bits < b.ia) b.ia = bits; }
    if (AGG == 2) { if (xd > b.dmm) b.dmm = xd; if (bits > b.ia) b.ia = bits; }
  }
  if (AGG == 4) wf_push(b.wf, xd);
}

template <int AGG>
DEVI void ffinalize(const DecodeArgs& a, const FBucket& b, uint64_t eidx, uint64_t eo) {
  const int64_t ts = b.ref + (int64_t)udiv64_32(b.rel, b.n);  // Span.java:399 floor(sum/n)
  const bool allint = b.nflt == 0;
  int64_t v;
  if (allint) {
    if (AGG == 3) v = ldiv64_32(b.ia, b.n);
    else if (AGG == 4) v = d2l(wf_result(b.wf));
    else v = b.ia;
  } else {
    double d;
    if (AGG == 0) d = b.dsum;
    else if (AGG == 3) d = b.dsum / (double)(int32_t)b.n;
    else if (AGG == 4) d = wf_result(b.wf);
    else d = b.dmm;
    v = dbits(d);
  }
  a.e_ts[eo + eidx] = (uint32_t)ts;
  a.e_val[eo + eidx] = v;
  a.e_flt[eo + eidx] = !allint;
}

// INL: the spans this kernel cannot take go straight to the general code in
// the same wave (k_decode.hip) instead of a list for a second launch; for the
// short leftover lists of k_direct_scan / k_ds_spans (one launch fewer).
template <int AGG, bool DS, bool INL = false>
__global__ void __launch_bounds__(256, 3) k_decode_fast(DecodeArgs a, const uint32_t* ncells, const uint32_t* vlen) {
  __shared__ FastLds lds[4];
  __shared__ int64_t s_gbits[INL && DS ? 4 : 1][WAVE];
  __shared__ uint8_t s_gflt[INL && DS ? 4 : 1][WAVE];
  const int lane = lane_id();
  const int wib = threadIdx.x / WAVE;
  FastLds& L = lds[wib];
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  const uint32_t nspan = a.span_list ? *a.span_count : a.n_kept;
  for (uint32_t i = wave; i < nspan; i += nwaves) {
    const uint32_t k = a.span_list ? a.span_list[i] : i;
    const uint32_t s = a.kept[k];
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    bool general = a.sp_q1[s] >= 0 || a.sp_ovf_cell[s] >= 0;
    const uint64_t eo = a.e_off[k], cap = a.sp_cap[s];
    bool seq = (AGG == 1 || AGG == 2 || AGG == 4);
  restart:
    bool unsorted = false, anyf = false, anyi = false;
    uint64_t ecount = 0;   // DS: buckets emitted; no-DS: E points written
    int64_t prev_ts = -1;  // last cell ts of the previous chunk
    bool open = false;
    int64_t E = 0;         // end (first ts + interval) of the open bucket
    uint32_t kstride = 0;  // guessed bucket length (cells), 0 = unknown
    uint64_t cbase = 0;    // span cell index of the chunk start
    uint64_t last_head = 0;  // span cell index of the open bucket's head
    uint64_t r = r0;
    RowMeta m;
    if (!general) {
      m = row_meta(a, r, ncells, vlen);
      if (!m.ok) general = true;
    }
    if (!general) {
      // one chunk of loads in flight while the current chunk is processed
      // (two in flight needs occupancy 2 and measured 1.45x slower)
      uint32_t c0 = 0;
      ChunkRaw cur, nxt;
      load_chunk(a, m, c0, cur);
      for (;;) {
        RowMeta nm = m;
        uint32_t nc0 = c0 + FCH;
        uint64_t nr = r;
        bool more = true;
        if (nc0 >= m.nc) {
          nr = r + 1;
          nc0 = 0;
          if (nr < r1) {
            nm = row_meta(a, nr, ncells, vlen);
            if (!nm.ok) { general = true; break; }
          } else {
            more = false;
          }
        }
        if (more) load_chunk(a, nm, nc0, nxt);
        const bool span_end = !more;
        // ---- decode the current chunk ----
        const uint32_t nv = min((uint32_t)FCH, m.nc - c0);        // valid cells
        const int64_t start_rel = a.start - (int64_t)m.base;      // E cells: dt >= start_rel
        uint32_t dt[4];
        int64_t bits[4];
        bool lenbad = false, ord = false, fl_any = false, int_any = false;
        uint32_t emask4 = 0, fmask4 = 0;  // per-lane 4-bit masks
        int first_e = 4;
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t c = c0 + 4 * lane + j;
          const bool valid = c < m.nc;
          const uint32_t q = qual_j(cur, j);
          dt[j] = q >> 4;
          const bool isf = (q & 8) != 0;
          lenbad |= valid && ((q & 7) + 1) != m.w;
          bits[j] = value_j(cur, j, m.w, isf);
          const bool ine = valid && (int64_t)dt[j] >= start_rel;
          if (ine) { emask4 |= 1u << j; if (first_e == 4) first_e = j; }
          if (ine && isf) fmask4 |= 1u << j;
          fl_any |= ine && isf;
          int_any |= ine && !isf;
          if (j > 0) ord |= valid && dt[j] <= dt[j - 1];
        }
        if (ballot(lenbad)) { general = true; break; }
        {
          const int lastj = (int)min(3u, nv > 4u * lane ? nv - 1 - 4u * lane : 0u);
          const uint32_t lastdt = lastj == 0 ? dt[0] : lastj == 1 ? dt[1] : lastj == 2 ? dt[2] : dt[3];
          int64_t pl = (int64_t)shfl_up_u32(lastdt, 1) + m.base;
          if (lane == 0) pl = prev_ts;
          ord |= 4u * lane < nv && (int64_t)m.base + dt[0] <= pl;
          if (ballot(ord)) unsorted = true;
          prev_ts = (int64_t)m.base + readlane_u32(lastdt, (int)((nv - 1) >> 2));
        }
        const uint64_t elanes = ballot(emask4 != 0);
        const bool has_f = ballot(fl_any) != 0;
        if (DS && has_f && !seq) { seq = true; goto restart; }
        anyf |= has_f;
        anyi |= ballot(int_any) != 0;
        if (!elanes) {  // whole chunk before start
          if (span_end) break;
          cbase += nv;
          cur = nxt; c0 = nc0; r = nr; m = nm;
          continue;
        }
        // first E cell of the chunk: E cells are a suffix of the valid cells
        const int fel = __builtin_ctzll(elanes);
        const int fe = 4 * fel + (int)readlane_u32((uint32_t)first_e, fel);
        if (!DS) {
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if (emask4 & (1u << j)) {
              const uint64_t e = ecount + (uint64_t)(4 * lane + j - fe);
              a.e_ts[eo + e] = m.base + dt[j];
              a.e_val[eo + e] = bits[j];
              a.e_flt[eo + e] = (fmask4 >> j) & 1;
            }
          }
          ecount += nv - (uint32_t)fe;
        } else {
          const int le = (int)nv - 1;
          // ---- DPP prefix sums over the chunk's E cells -> LDS ----
          uint32_t pt = 0, pf = 0;
          uint64_t pv = 0;
          uint32_t pti[4], pfi[4];
          uint64_t pvi[4];
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if (emask4 & (1u << j)) { pt += dt[j]; pv += (uint64_t)bits[j]; pf += (fmask4 >> j) & 1; }
            pti[j] = pt; pvi[j] = pv; pfi[j] = pf;
          }
          const uint32_t xt = wave_incl_scan_u32_dpp(pt) - pt;
          const uint64_t xv = wave_incl_scan_u64_dpp(pv) - pv;
          uint32_t xf = 0;
          if (seq) xf = wave_incl_scan_u32_dpp(pf) - pf;
          *(uint4*)&L.pt[4 * lane] = make_uint4(pti[0] + xt, pti[1] + xt, pti[2] + xt, pti[3] + xt);
          *(uint4*)&L.dtv[4 * lane] = make_uint4(dt[0], dt[1], dt[2], dt[3]);
          {
            ulonglong2 v01, v23;
            v01.x = pvi[0] + xv; v01.y = pvi[1] + xv; v23.x = pvi[2] + xv; v23.y = pvi[3] + xv;
            *(ulonglong2*)&L.pv[4 * lane] = v01;
            *(ulonglong2*)&L.pv[4 * lane + 2] = v23;
          }
          if (seq) {
            *(uint4*)&L.pf[4 * lane] = make_uint4(pfi[0] + xf, pfi[1] + xf, pfi[2] + xf, pfi[3] + xf);
            longlong2 b01, b23;
            b01.x = bits[0]; b01.y = bits[1]; b23.x = bits[2]; b23.y = bits[3];
            *(longlong2*)&L.bits[4 * lane] = b01;
            *(longlong2*)&L.bits[4 * lane + 2] = b23;
            *(uint32_t*)&L.flt[4 * lane] = (fmask4 & 1) | ((fmask4 & 2) << 7) | ((fmask4 & 4) << 14) |
                                            ((fmask4 & 8) << 21);
          }
          wave_lds_sync();
          // ---- bucket heads (Span.java:389-398) ----
          const int64_t base = (int64_t)m.base;
          const int64_t tsfe = base + (int64_t)L.dtv[fe];
          const bool cont = open && tsfe < E;
          if (open && !cont) {  // carried bucket closed exactly at the chunk start
            if (lane == 0 && ecount < cap) ffinalize<AGG>(a, L.carry, ecount, eo);
            ecount++;
            open = false;
          }
          // first new-bucket end after fe
          const int64_t E0 = cont ? E : tsfe + a.interval;
          int nh = 0;         // heads written after heads[0] = fe
          int64_t Eend = E0;  // end of the last bucket started in this chunk
          bool spec_ok = false;
          if (kstride > 0) {
            // guess: next head p = (last head + k) or fe + k, then stride k
            const int64_t p_span = cont ? (int64_t)(last_head + kstride) : (int64_t)(cbase + fe + kstride);
            const int64_t p = p_span - (int64_t)cbase;
            const int64_t g = p + (int64_t)lane * kstride;   // this lane's guessed head
            const int m_n = p > le ? 0 : (int)min((int64_t)64, (le - p) / (int64_t)kstride + 1);
            // structurally possible? (uniform)
            if (p > fe && m_n < WAVE) {
              const bool mine = lane < m_n;
              bool bad = false;
              if (mine) {
                const int64_t prevend = lane == 0 ? E0 : base + (int64_t)L.dtv[g - kstride] + a.interval;
                const int64_t tg = base + (int64_t)L.dtv[g], tgm = base + (int64_t)L.dtv[g - 1];
                bad = !(tg >= prevend && tgm < prevend);
              }
              // tail: cells after the last head stay in its bucket
              const int64_t lastend =
                  m_n == 0 ? E0 : base + (int64_t)L.dtv[p + (int64_t)(m_n - 1) * kstride] + a.interval;
              bad = bad || (base + (int64_t)L.dtv[le] >= lastend);
              if (ballot(bad) == 0) {
                spec_ok = true;
                if (mine) L.heads[1 + lane] = (uint16_t)g;
                nh = m_n;
                Eend = lastend;
              }
            }
          }
          if (!spec_ok) {
            // serial ballot chain: one VALU compare per head
            const int lastj = 31 - __builtin_clz(emask4 | 1u);
            const uint32_t ldt = lastj == 0 ? dt[0] : lastj == 1 ? dt[1] : lastj == 2 ? dt[2] : dt[3];
            int after = fe + 1;
            int64_t Ecur = E0;
            for (;;) {
              const int64_t x = Ecur - base;
              const uint32_t er = x <= 0 ? 0u : (x >= 0xFFFFFFFFll ? 0xFFFFFFFFu : (uint32_t)x);
              const uint64_t cand = ballot(emask4 != 0 && ldt >= er) & ~lanemask_lt(after >> 2) & elanes;
              if (!cand) break;
              const int Lh = __builtin_ctzll(cand);
              int c = -1;
#pragma unroll
              for (int j = 3; j >= 0; j--) {
                const int cj = 4 * Lh + j;
                if (cj >= after && cj <= le && L.dtv[cj] >= er) c = cj;
              }
              c = __builtin_amdgcn_readfirstlane(c);
              if (c < 0) { after = 4 * Lh + 4; continue; }
              if (nh == WAVE - 1) { nh = -1; break; }  // one lane per segment: at most 64
              if (lane == 0) L.heads[1 + nh] = (uint16_t)c;
              nh++;
              Ecur = base + (int64_t)L.dtv[c] + a.interval;
              after = c + 1;
            }
            if (nh < 0) { general = true; break; }  // > 64 buckets in one chunk
            Eend = Ecur;
          }
          if (lane == 0) { L.heads[0] = (uint16_t)fe; L.heads[1 + nh] = (uint16_t)(le + 1); }
          wave_lds_sync();
          const int nseg = nh + 1;
          // stride for the next chunk: the last complete new bucket's length
          if (nseg >= 3) kstride = (uint32_t)(L.heads[nseg - 1] - L.heads[nseg - 2]);
          else if (nseg == 2 && !cont) kstride = (uint32_t)(L.heads[1] - L.heads[0]);
          else if (nseg == 2 && cont) kstride = (uint32_t)(cbase + L.heads[1] - last_head);
          // ---- one lane per segment ----
          FBucket b;
          b.n = 0;
          if (lane < nseg) {
            const int sa = L.heads[lane];
            const int sb = (int)L.heads[lane + 1] - 1;
            const uint32_t n = (uint32_t)(sb - sa + 1);
            const uint32_t ptb = L.pt[sb], pta = sa > 0 ? L.pt[sa - 1] : 0u;
            const uint32_t dta = L.dtv[sa];
            b.n = n;
            b.ref = base + dta;
            b.rel = (uint64_t)((ptb - pta) - n * dta);
            b.nflt = seq ? L.pf[sb] - (sa > 0 ? L.pf[sa - 1] : 0u) : 0u;
            b.ia = (int64_t)(L.pv[sb] - (sa > 0 ? L.pv[sa - 1] : 0ull));
            b.dsum = 0; b.dmm = 0; wf_init(b.wf);
            const bool c0seg = lane == 0 && cont;
            const int64_t ia_pref = b.ia;
            if (seq) {
              bool first = true;
              if (c0seg) { b.dsum = L.carry.dsum; b.dmm = L.carry.dmm; b.wf = L.carry.wf; b.ia = L.carry.ia; first = false; }
              for (int i = sa; i <= sb; i++) {
                fpush<AGG>(b, L.bits[i], L.flt[i] != 0, first);
                first = false;
              }
            }
            if (AGG == 0 || AGG == 3) b.ia = ia_pref;
            if (c0seg) {
              // continue the carried bucket: re-base the chunk part on its ref
              const FBucket& cb = L.carry;
              b.rel = cb.rel + b.rel + (uint64_t)n * (uint64_t)(b.ref - cb.ref);
              b.ref = cb.ref;
              b.n += cb.n;
              b.nflt += cb.nflt;
              if (AGG == 0 || AGG == 3) b.ia = ladd(cb.ia, b.ia);
            }
          }
          const int nclosed = span_end ? nseg : nseg - 1;
          if (lane < nclosed && ecount + lane < cap) ffinalize<AGG>(a, b, ecount + lane, eo);
          ecount += nclosed;
          wave_lds_sync();
          if (!span_end) {
            if (lane == nseg - 1) L.carry = b;
            if (nseg > 1 || !cont) last_head = cbase + L.heads[nseg - 1];
            E = Eend;
            open = true;
          } else {
            open = false;
          }
          wave_lds_sync();
        }
        if (span_end) break;
        cbase += nv;
        cur = nxt; c0 = nc0; r = nr; m = nm;
      }
      if (!general) {
        if (lane == 0) {
          a.e_len[k] = (uint32_t)(ecount < cap ? ecount : cap);
          if (ecount > cap) err_raise(a.err, 2, a.span0 + s, -4 /*E_CAPACITY*/);
          a.e_bad[k] = -1;
          if (unsorted) err_raise(a.err, 2, a.span0 + s, -8 /*E_UNSORTED*/);
          if (anyf) atomicOr(&a.gflags[0], 1u);
          if (anyi) atomicOr(&a.gflags[1], 1u);
        }
        continue;
      }
    }
    // ---- fallback: the general code rewrites the span's E ----
    if (INL) {
      if (DS) span_ds_general<AGG>(a, k, s_gbits[INL && DS ? wib : 0], s_gflt[INL && DS ? wib : 0]);
      else span_nods_general(a, k);
    } else if (lane == 0) {  // (queued for the general kernel)
      a.fb_list[atomicAdd(a.fb_count, 1u)] = k;
    }
  }
}

}  // namespace tsdb
