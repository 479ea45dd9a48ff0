// k_decode_fast.hip — the HBM-streaming decode(+downsample) kernel for spans
// whose rows have one value width (8-byte longs / doubles, 4-byte floats /
// ints): the reference's write paths produce exactly these rows
// (IncomingDataPoints.java:273-282, TSDB.java:285,321). Same semantics as
// k_decode.hip (RowSeq.Iterator + Span.DownsamplingIterator); any span that
// breaks the preconditions (mixed widths, dropped rows, quirk Q1, the short
// overflow, unaligned rows) is handed to the general per-span routine.
//
// Per wave-iteration a chunk of 256 cells of one row: lane l owns cells
// 4l..4l+3 (8-byte qualifier load, 16/32-byte value loads), and the next
// chunk's loads are issued before the current one is processed.
// Downsampling: greedy bucket heads come from a ballot chain over the 256
// cells; bucket count / timestamp sum / float count / integer sum are
// differences of chunk prefix sums staged in LDS (exact integer arithmetic);
// order-dependent parts (double sums of float buckets, min/max, dev) run one
// lane per bucket over the LDS-staged values in point order (exact).
#pragma once
#include "dev_common.h"
#include "k_decode.hip"

namespace tsdb {

#define FCH 256  // cells per chunk

struct FastLds {
  uint64_t pv[FCH];   // inclusive prefix of integer values (wrapping)
  int64_t bits[FCH];  // decoded value bits (ordered pass)
  uint32_t pt[FCH];   // inclusive prefix of ts deltas within the row
  uint16_t pf[FCH];   // inclusive prefix of float cells
  uint8_t flt[FCH];
  uint16_t heads[FCH + 2];
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
DEVI void seq_push_both(Bucket& b, int64_t bits, bool flt, bool first) {
  const double xd = to_double(bits, flt);
  if (first) { b.dsum = xd; b.dmm = xd; b.ia = bits; }
  else {
    b.dsum += xd;
    if (AGG == 1) { if (xd < b.dmm) b.dmm = xd; if (bits < b.ia) b.ia = bits; }
    if (AGG == 2) { if (xd > b.dmm) b.dmm = xd; if (bits > b.ia) b.ia = bits; }
  }
  if (AGG == 4) wf_push(b.wf, xd);
}

template <int AGG, bool DS>
__global__ void __launch_bounds__(256, 3) k_decode_fast(DecodeArgs a, const uint32_t* ncells, const uint32_t* vlen) {
  __shared__ FastLds lds[4];
  const int lane = lane_id();
  const int wib = threadIdx.x / WAVE;
  FastLds& L = lds[wib];
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) / WAVE;
  const uint32_t nwaves = gridDim.x * blockDim.x / WAVE;
  for (uint32_t k = wave; k < a.n_kept; k += nwaves) {
    const uint32_t s = a.kept[k];
    const uint64_t r0 = a.span_row_start[s], r1 = a.span_row_start[s + 1];
    bool general = a.sp_q1[s] >= 0 || a.sp_ovf_cell[s] >= 0;
    const uint64_t eo = a.e_off[k], cap = a.sp_cap[s];
    bool seq = (AGG == 1 || AGG == 2 || AGG == 4);
  restart:
    bool unsorted = false, anyf = false, anyi = false;
    uint64_t ecount = 0;   // DS: buckets emitted; no-DS: E points written
    uint64_t cell = 0;     // span cell index of the chunk start
    int64_t prev_ts = -1;
    bool open = false;
    Bucket cb;
    cb.end = 0; cb.n = 0; cb.nflt = 0; cb.tssum = 0; cb.ia = 0; cb.dsum = 0; cb.dmm = 0;
    wf_init(cb.wf); cb.bad = false;
    uint64_t r = r0;
    RowMeta m;
    if (!general) {
      m = row_meta(a, r, ncells, vlen);
      if (!m.ok) general = true;
    }
    if (!general) {
      uint32_t c0 = 0;
      ChunkRaw cur, nxt;
      load_chunk(a, m, c0, cur);
      for (;;) {
        // ---- position and prefetch of the next chunk ----
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
        int64_t ts[4], bits[4];
        bool valid[4], ine[4], flt[4];
        bool lenbad = false, ord = false;
        uint32_t dt[4];
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const uint32_t c = c0 + 4 * lane + j;
          valid[j] = c < m.nc;
          const uint32_t q = qual_j(cur, j);
          dt[j] = q >> 4;
          ts[j] = valid[j] ? (int64_t)m.base + dt[j] : INT64_MAX;
          flt[j] = valid[j] && (q & 8);
          lenbad |= valid[j] && ((q & 7) + 1) != m.w;
          bits[j] = valid[j] ? value_j(cur, j, m.w, (q & 8) != 0) : 0;
          ine[j] = valid[j] && ts[j] >= a.start;
          if (j > 0) ord |= valid[j] && ts[j] <= ts[j - 1];
        }
        if (ballot(lenbad)) { general = true; break; }
        {
          const int64_t lastv = valid[3] ? ts[3] : valid[2] ? ts[2] : valid[1] ? ts[1] : ts[0];
          int64_t pl = (int64_t)shfl_up_u64((uint64_t)lastv, 1);
          if (lane == 0) pl = prev_ts;
          ord |= valid[0] && ts[0] <= pl;
          if (ballot(ord)) unsorted = true;
          const uint32_t nv = min((uint32_t)FCH, m.nc - c0);
          const int ll = (int)((nv - 1) >> 2), lj = (int)((nv - 1) & 3);
          prev_ts = (int64_t)readlane_u64((uint64_t)(lj == 0 ? ts[0] : lj == 1 ? ts[1] : lj == 2 ? ts[2] : ts[3]), ll);
        }
        const uint64_t fm = ballot(flt[0] && ine[0]) | ballot(flt[1] && ine[1]) | ballot(flt[2] && ine[2]) |
                            ballot(flt[3] && ine[3]);
        const uint64_t em = ballot(ine[0]) | ballot(ine[1]) | ballot(ine[2]) | ballot(ine[3]);
        if (DS && fm && !seq) { seq = true; goto restart; }
        anyf |= fm != 0;
        {
          const bool ii = (ine[0] && !flt[0]) || (ine[1] && !flt[1]) || (ine[2] && !flt[2]) || (ine[3] && !flt[3]);
          anyi |= ballot(ii) != 0;
        }
        if (!DS) {
          // ---- plain E write: E index = cell index - cells before start ----
          const uint32_t nskip_c = __popcll(ballot(valid[0] && !ine[0])) + __popcll(ballot(valid[1] && !ine[1])) +
                                   __popcll(ballot(valid[2] && !ine[2])) + __popcll(ballot(valid[3] && !ine[3]));
          // cells < start are a prefix of the span; ecount = E points so far
          const uint32_t in_chunk_e0 = nskip_c;  // first E cell index in the chunk
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if (ine[j]) {
              const uint64_t e = ecount + (4 * lane + j) - in_chunk_e0;
              a.e_ts[eo + e] = (uint32_t)ts[j];
              a.e_val[eo + e] = bits[j];
              a.e_flt[eo + e] = flt[j];
            }
          }
          ecount += (uint64_t)min((uint32_t)FCH, m.nc - c0) - nskip_c;
        } else if (em) {
          // ---- E cells of this chunk: [fe, le] (a suffix of the valid cells) ----
          const uint32_t nv = min((uint32_t)FCH, m.nc - c0);
          const int le = (int)nv - 1;
          uint32_t nskip_c = __popcll(ballot(valid[0] && !ine[0])) + __popcll(ballot(valid[1] && !ine[1])) +
                             __popcll(ballot(valid[2] && !ine[2])) + __popcll(ballot(valid[3] && !ine[3]));
          const int fe = (int)nskip_c;
          // ---- prefix sums over the chunk (E cells only) -> LDS ----
          uint32_t pt = 0, pf = 0;
          uint64_t pv = 0;
          uint32_t pti[4], pfi[4];
          uint64_t pvi[4];
#pragma unroll
          for (int j = 0; j < 4; j++) {
            if (ine[j]) { pt += dt[j]; pf += flt[j] ? 1u : 0u; pv += (uint64_t)bits[j]; }
            pti[j] = pt; pfi[j] = pf; pvi[j] = pv;
          }
          const uint32_t xt = wave_incl_scan_u32(pt) - pt;
          const uint32_t xf = wave_incl_scan_u32(pf) - pf;
          const uint64_t xv = wave_incl_scan_u64(pv) - pv;
#pragma unroll
          for (int j = 0; j < 4; j++) {
            const int c = 4 * lane + j;
            L.pt[c] = pti[j] + xt;
            L.pf[c] = (uint16_t)(pfi[j] + xf);
            L.pv[c] = pvi[j] + xv;
            if (seq) { L.bits[c] = bits[j]; L.flt[c] = flt[j]; }
          }
          // ---- greedy bucket chain (Span.java:389-398) ----
          const int fl = fe >> 2, fj = fe & 3;
          const int64_t tsfe = (int64_t)readlane_u64((uint64_t)(fj == 0 ? ts[0] : fj == 1 ? ts[1] : fj == 2 ? ts[2] : ts[3]), fl);
          bool cont = open && tsfe < cb.end;
          if (open && !cont) {  // carried bucket closed exactly at the chunk start
            if (lane == 0 && ecount < cap) finalize_bucket<AGG>(a, cb, ecount, eo);
            ecount++;
            open = false;
          }
          int nh = 0;
          if (cont) { if (lane == 0) L.heads[0] = (uint16_t)fe; nh = 1; }
          int64_t E = cont ? cb.end : INT64_MIN;
          int after = fe;
          for (;;) {
            int fjj = 4;
#pragma unroll
            for (int j = 3; j >= 0; j--)
              if (ine[j] && ts[j] >= E && 4 * lane + j >= after) fjj = j;
            const uint64_t mm = ballot(fjj < 4);
            if (!mm) break;
            const int Lh = __builtin_ctzll(mm);
            const int J = (int)readlane_u32((uint32_t)fjj, Lh);
            const int c = 4 * Lh + J;
            const int64_t tsv = (int64_t)readlane_u64((uint64_t)(J == 0 ? ts[0] : J == 1 ? ts[1] : J == 2 ? ts[2] : ts[3]), Lh);
            if (lane == 0) L.heads[nh] = (uint16_t)c;
            nh++;
            E = tsv + a.interval;
            after = c + 1;
          }
          if (lane == 0) L.heads[nh] = (uint16_t)(le + 1);
          wave_lds_sync();
          const int nseg = nh;
          // ---- one lane per segment ----
          Bucket b;
          int sa = 0, sb = -1;
          if (lane < nseg) {
            sa = L.heads[lane];
            sb = (int)L.heads[lane + 1] - 1;
            const uint32_t n = (uint32_t)(sb - sa + 1);
            b.n = n;
            const uint32_t ptb = L.pt[sb], pta = sa > 0 ? L.pt[sa - 1] : 0u;
            b.tssum = (uint64_t)n * m.base + (uint64_t)(ptb - pta);
            b.nflt = (uint32_t)L.pf[sb] - (sa > 0 ? (uint32_t)L.pf[sa - 1] : 0u);
            b.ia = (int64_t)(L.pv[sb] - (sa > 0 ? L.pv[sa - 1] : 0ull));
            b.bad = false; b.end = 0; b.dsum = 0; b.dmm = 0; wf_init(b.wf);
            const int64_t ia_pref = b.ia;  // integer sum of the segment (prefixes)
            if (seq) {
              bool first = true;
              if (lane == 0 && cont) { b.dsum = cb.dsum; b.dmm = cb.dmm; b.wf = cb.wf; b.ia = cb.ia; first = false; }
              for (int i = sa; i <= sb; i++) {
                seq_push_both<AGG>(b, L.bits[i], L.flt[i] != 0, first);
                first = false;
              }
            }
            if (AGG == 0 || AGG == 3) b.ia = ia_pref;
            if (lane == 0 && cont) {
              b.n += cb.n; b.nflt += cb.nflt; b.tssum += cb.tssum;
              if (AGG == 0 || AGG == 3) b.ia = ladd(cb.ia, b.ia);
            }
          }
          const int nclosed = span_end ? nseg : nseg - 1;
          if (lane < nclosed && ecount + lane < cap) finalize_bucket<AGG>(a, b, ecount + lane, eo);
          ecount += nclosed;
          if (!span_end && nseg > 0) {
            const int j = nseg - 1;
            cb.n = readlane_u32(b.n, j);
            cb.nflt = readlane_u32(b.nflt, j);
            cb.tssum = readlane_u64(b.tssum, j);
            cb.ia = (int64_t)readlane_u64((uint64_t)b.ia, j);
            cb.dsum = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.dsum), j));
            cb.dmm = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.dmm), j));
            cb.wf.n = (int64_t)readlane_u64((uint64_t)b.wf.n, j);
            cb.wf.mean = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.wf.mean), j));
            cb.wf.var = bitsd((int64_t)readlane_u64((uint64_t)dbits(b.wf.var), j));
            cb.end = E;
            open = true;
          } else {
            open = false;
          }
          wave_lds_sync();
        }
        if (span_end) break;
        // advance
        cell += m.nc > c0 + FCH ? FCH : (m.nc - c0);
        cur = nxt;
        c0 = nc0;
        r = nr;
        m = nm;
      }
      if (!general) {
        if (lane == 0) {
          a.e_len[k] = (uint32_t)(ecount < cap ? ecount : cap);
          if (ecount > cap) atomicMin(a.err, -4 /*E_CAPACITY*/);
          a.e_bad[k] = -1;
          if (unsorted) atomicMin(a.err, -8 /*E_UNSORTED*/);
          if (anyf) atomicOr(&a.gflags[0], 1u);
          if (anyi) atomicOr(&a.gflags[1], 1u);
        }
        continue;
      }
    }
    // ---- fallback: queue the span for the general kernel (rewrites its E) ----
    if (lane == 0) a.fb_list[atomicAdd(a.fb_count, 1u)] = k;
  }
}

}  // namespace tsdb
